#!/bin/bash
# Round-2 session e: conv/wgrad A/B, the GPU suite, bench, kernel-trace profile.
TAG=${1:-r2e}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
run() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -v amdgpu.ids $OUT/$name.log | tail -${TAILN:-12}
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name"; exit $rc; fi
  return 0
}
run resnet 300 python -u -m pytest tests/test_resnet_gpu.py -x -q --timeout 120 --timeout-method thread
TAILN=12 run conv_v0 200 env MER_CONV_VEC=0 MER_WGRAD_VARIANT=2 python -u tools/bench_conv.py --fused --variants=2
TAILN=12 run conv_v1 200 python -u tools/bench_conv.py --fused --variants=2
run bench 300 python -u bench.py --no-cpu-baseline
run pytest 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python $OLDPWD/bench.py --steps 10 --warmup 3 --probe-steps 5 --no-cpu-baseline > $OUT/prof.log 2>&1); echo "== prof rc=$?"
echo SESSION_DONE
