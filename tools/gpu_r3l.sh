#!/bin/bash
OUT=$PWD/gpurun_out/r3l
mkdir -p $OUT; rm -f $OUT/summary.log
for cfg in "0 auto before_adam" "0 auto before_trunk_bwd" "0 auto before_head_bwd" "0 auto before_adam" "0 auto before_trunk_bwd" "0 auto before_head_bwd"; do
  tag=$(echo $cfg | tr ' ' '_')
  timeout -k 10 200 python -u tools/diag_grads.py $cfg > $OUT/g_$tag.log 2>&1 || exit 1
  echo "== $cfg" >> $OUT/summary.log
  grep "^step [345]" $OUT/g_$tag.log | cut -c1-60 >> $OUT/summary.log
done
