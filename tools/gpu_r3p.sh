#!/bin/bash
OUT=$PWD/gpurun_out/r3p
mkdir -p $OUT; rm -f $OUT/summary.log
timeout -k 10 300 python -u tools/diag_concurrent.py > $OUT/c.log 2>&1 || exit 1
grep "WavLM replay" $OUT/c.log >> $OUT/summary.log
for i in 1 2; do
  timeout -k 10 200 python -u tools/diag_grads.py 0 auto none > $OUT/g$i.log 2>&1 || exit 1
  echo "== late path run $i" >> $OUT/summary.log; grep "^step [345]" $OUT/g$i.log | cut -c1-60 >> $OUT/summary.log
done
timeout -k 10 600 python -u -m pytest tests/test_train_epoch_gpu.py tests/test_xattn_fused_gpu.py tests/test_head_gpu.py tests/test_dp_gpu.py -m gpu -q --timeout 500 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "TESTS_EXIT $rc" >> $OUT/summary.log; tail -4 $OUT/tests.log >> $OUT/summary.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python -u tools/bench_head.py >> $OUT/summary.log 2>&1
