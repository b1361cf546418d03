#!/bin/bash
# Round-2 session j: stage-2 dropout tests, full GPU suite, benches (headline + stage 2), kernel-trace profile.
TAG=${1:-r2j}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
run() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -v amdgpu.ids $OUT/$name.log | tail -${TAILN:-6} | cut -c1-400
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name"; exit $rc; fi
  return 0
}
TAILN=40 run stage2 400 python -u -m pytest tests/test_wavlm_stage2_gpu.py -x -v --timeout 200 --timeout-method thread
run pytest 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
run bench 300 python -u bench.py --no-cpu-baseline
run bench_stage2 300 python -u bench.py --no-cpu-baseline --wavlm-unfreeze 2 --probe-steps 0 --probe-launches 0
echo SESSION_DONE
