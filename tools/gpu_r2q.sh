#!/bin/bash
# Round-2 session q: training loop on a high-priority stream vs normal (same box, alternating).
TAG=${1:-r2q}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
run() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -v amdgpu.ids $OUT/$name.log | tail -1 | cut -c1-200
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name"; exit $rc; fi
  return 0
}
for i in 1 2; do
  run hi$i 200 python -u bench.py --no-cpu-baseline --probe-steps 0 --probe-launches 0 --stream-priority high
  run lo$i 200 python -u bench.py --no-cpu-baseline --probe-steps 0 --probe-launches 0
done
echo SESSION_DONE
