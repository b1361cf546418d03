#!/bin/bash
# Round-2 session d: GEMM calibration vs hipBLASLt on the WavLM linears, conv/wgrad A/B (prefetch depth, epilogue).
TAG=${1:-r2d}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
run() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; cat $OUT/$name.log | grep -v amdgpu.ids | tail -40
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name"; exit $rc; fi
  return 0
}
run resnet 300 python -u -m pytest tests/test_resnet_gpu.py -x -q --timeout 120 --timeout-method thread
run gemm 300 python -u tools/bench_gemm.py --shapes=qkv,ffn1,ffn2,out_proj --variants=13,12,9,7,4 --blas
run conv_w2 200 env MER_CONV_VEC=0 python -u tools/bench_conv.py --fused --variants=2 --wgrad-variants=2,3
run conv_w3 200 python -u tools/bench_conv.py --fused --variants=2 --wgrad-variants=3
run bench 300 python -u bench.py --no-cpu-baseline
echo SESSION_DONE
