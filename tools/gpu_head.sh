#!/bin/bash
# fused-head parity tests + isolated head timing + its per-kernel profile.  Usage: bash tools/gpu_head.sh TAG
TAG=${1:-head}
R=$PWD
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
bash tools/gpu_tests.sh $TAG "tests/test_xattn_fused_gpu.py tests/test_head_gpu.py" || exit 1
grep -E "worst" $OUT/focus.log | sed 's/.*\] //'
timeout -k 10 200 python -u tools/bench_head.py > $OUT/head.log 2>&1 || { tail $OUT/head.log; exit 1; }
grep -E "fused" $OUT/head.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python $R/tools/bench_head.py --iters 50 > $OUT/prof.log 2>&1
echo "PROF_EXIT $?"
cd $R && python tools/kstats.py $OUT/prof/run_kernel_stats.csv 1 40 | grep -E "xh_|total"
timeout -k 10 120 python -u tools/xt_phases.py run 2>&1 | grep -v amdgpu.ids
