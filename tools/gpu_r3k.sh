#!/bin/bash
OUT=$PWD/gpurun_out/r3k
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_xattn_fused_gpu.py tests/test_head_gpu.py tests/test_round2_features_gpu.py tests/test_int8_gpu.py tests/test_graphs_gpu.py -m gpu -q --timeout 300 --timeout-method thread -s > $OUT/tests.log 2>&1
rc=$?; echo "EXIT $rc" >> $OUT/tests.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python -u tools/bench_head.py > $OUT/head.log 2>&1
rc=$?; echo "EXIT $rc" >> $OUT/head.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/diag_graph_wait.py > $OUT/g.log 2>&1
echo "EXIT $?" >> $OUT/g.log
