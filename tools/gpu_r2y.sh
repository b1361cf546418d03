#!/bin/bash
# One-launch BN fold+finalize: resnet GPU tests, full suite, same-box bench A/B (MER_BN_FUSED_FINALIZE 0 / 1).
R=$PWD; OUT=$R/gpurun_out/r2y; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_resnet_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest_resnet.log 2>&1; rc=$?; tail -4 $OUT/pytest_resnet.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -4 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1 0 1; do
  MER_BN_FUSED_FINALIZE=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --probe-steps 0 > $OUT/bench_$v.log 2>&1; rc=$?
  echo "== fused=$v rc=$rc"; tail -1 $OUT/bench_$v.log | cut -c100-200; [ $rc -eq 0 ] || exit $rc
done
