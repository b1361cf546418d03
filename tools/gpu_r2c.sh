#!/bin/bash
# Round-2 session c: conv epilogue A/B, then the GPU suite, bench and a kernel-trace profile.
#   bash tools/gpu_r2c.sh TAG [quick]
TAG=${1:-r2c}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
run() {  # name timeout cmd...   (stops the session on a fault / abort / timeout)
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -4 $OUT/$name.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name"; exit $rc; fi
  return 0
}
run resnet 300 python -u -m pytest tests/test_resnet_gpu.py -x -q --timeout 120 --timeout-method thread
run conv_vec0 200 env MER_CONV_VEC=0 python -u tools/bench_conv.py --fused --no-wgrad --variants=2
run conv_vec1 200 python -u tools/bench_conv.py --fused --no-wgrad --variants=2
cat $OUT/conv_vec0.log $OUT/conv_vec1.log
if [ "$2" == "quick" ]; then echo SESSION_DONE; exit 0; fi
run pytest 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run bench 300 python -u bench.py --no-cpu-baseline
tail -1 $OUT/bench.log
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python $OLDPWD/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/prof.log 2>&1); echo "== prof rc=$?"
echo SESSION_DONE
