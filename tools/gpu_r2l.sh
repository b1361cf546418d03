#!/bin/bash
# Round-2 session l: deep-ring wgrad (32-pixel K-steps) correctness + A/B.
TAG=${1:-r2l}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
run() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -v amdgpu.ids $OUT/$name.log | tail -${TAILN:-12} | cut -c1-400
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name"; exit $rc; fi
  return 0
}
run wgradtest 300 python -u -m pytest tests/test_resnet_gpu.py -x -q --timeout 120 --timeout-method thread -k "wgrad or variants"
run conv 200 python -u tools/bench_conv.py --variants= --wgrad-variants=4,6,7
run conv_fwd 200 python -u tools/bench_conv.py --fused --no-wgrad --variants=2,4,5
echo SESSION_DONE
