#!/bin/bash
# Round-2 session f: stream-overlap accounting and same-box A/B benches.
TAG=${1:-r2f}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
run() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -v amdgpu.ids $OUT/$name.log | tail -${TAILN:-3} | cut -c1-400
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name"; exit $rc; fi
  return 0
}
run overlap 200 python -u tools/overlap_probe.py
run bench_a 200 python -u bench.py --no-cpu-baseline --probe-steps 0 --probe-launches 0
run bench_noprefetch 200 python -u bench.py --no-cpu-baseline --probe-steps 0 --probe-launches 0 --no-prefetch
run bench_old 200 env MER_CONV_VEC=0 MER_WGRAD_VARIANT=2 python -u bench.py --no-cpu-baseline --probe-steps 0 --probe-launches 0
run bench_b 200 python -u bench.py --no-cpu-baseline --probe-steps 0 --probe-launches 0
echo SESSION_DONE
