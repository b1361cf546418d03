#!/bin/bash
# W (grouped head weight gradients) vs rows per workgroup: standalone head timing + kernel trace per setting.
OUT=$PWD/gpurun_out/${1:-wrows}; shift
mkdir -p $OUT; R=$PWD
cd /tmp && export TMPDIR=/tmp && cd $R
for r in "$@"; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/p$r -o head -- python tools/bench_head.py --iters 50 --fused-only 1 --wgrad-rows $r > $OUT/head_$r.log 2>&1 || exit 1
  echo "rows $r: $(grep fused $OUT/head_$r.log) | $(grep -h 'xh_wgrad\|xh_wfold' $OUT/p$r/head_kernel_stats.csv | cut -d, -f1,4 | tr '\n' ' ')"
done
