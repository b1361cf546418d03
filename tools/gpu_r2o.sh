#!/bin/bash
# Round-2 session o: parity-class order (longest first) -- tests + conv A/B + bench.
TAG=${1:-r2o}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
run() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -v amdgpu.ids $OUT/$name.log | tail -${TAILN:-12} | cut -c1-300
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name"; exit $rc; fi
  return 0
}
run resnet 300 python -u -m pytest tests/test_resnet_gpu.py -x -q --timeout 120 --timeout-method thread
run conv 200 python -u tools/bench_conv.py --fused --no-wgrad --variants=2,5
TAILN=2 run bench 200 python -u bench.py --no-cpu-baseline --probe-steps 0 --probe-launches 0
echo SESSION_DONE
