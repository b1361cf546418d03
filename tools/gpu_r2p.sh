#!/bin/bash
# Round-2 session p: high-priority compute stream -- GPU suite + same-box bench A/B.
TAG=${1:-r2p}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
run() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -v amdgpu.ids $OUT/$name.log | tail -${TAILN:-2} | cut -c1-300
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name"; exit $rc; fi
  return 0
}
run pytest 800 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
run bench_hi1 200 python -u bench.py --no-cpu-baseline --probe-steps 0 --probe-launches 0
run bench_hi0 200 env MER_HIPRIO=0 python -u bench.py --no-cpu-baseline --probe-steps 0 --probe-launches 0
run bench_hi1b 200 python -u bench.py --no-cpu-baseline --probe-steps 0 --probe-launches 0
run bench_hi0b 200 env MER_HIPRIO=0 python -u bench.py --no-cpu-baseline --probe-steps 0 --probe-launches 0
echo SESSION_DONE
