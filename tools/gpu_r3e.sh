#!/bin/bash
# determinism bisect + head phase timing + isolated head timing
OUT=$PWD/gpurun_out/r3e
mkdir -p $OUT
timeout -k 10 400 python -u tools/diag_determinism.py 4 0,1,- 0,1,wavlm 0,1,trunk 0,1,head 1,1,- > $OUT/diag.log 2>&1
rc=$?; echo "DIAG_EXIT $rc" >> $OUT/diag.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/xt_phases.py run > $OUT/xt.log 2>&1
rc=$?; echo "XT_EXIT $rc" >> $OUT/xt.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/bench_head.py > $OUT/head.log 2>&1
echo "HEAD_EXIT $?" >> $OUT/head.log
