#!/bin/bash
OUT=$PWD/gpurun_out/r3o
mkdir -p $OUT; rm -f $OUT/summary.log
for kv in 1 0 1 0; do
  HIP_FORCE_DEV_KERNARG=$kv timeout -k 10 200 python -u tools/diag_grads.py 0 auto none > $OUT/g_k$kv.log 2>&1 || exit 1
  echo "== HIP_FORCE_DEV_KERNARG=$kv" >> $OUT/summary.log
  grep "^step [345]" $OUT/g_k$kv.log | cut -c1-60 >> $OUT/summary.log
done
timeout -k 10 600 python -u -m pytest tests/test_xattn_fused_gpu.py tests/test_head_gpu.py -m gpu -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "TESTS_EXIT $rc" >> $OUT/summary.log; tail -3 $OUT/tests.log >> $OUT/summary.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python -u tools/bench_head.py >> $OUT/summary.log 2>&1
