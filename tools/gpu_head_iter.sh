#!/bin/bash
# Head iteration: fused-head tests, phase stamps of a graph replay, standalone timing, kernel trace of the fused head.
#   bash tools/gpu_head_iter.sh TAG
TAG=${1:-head}
R=$PWD
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_head_gpu.py tests/test_xattn_fused_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/t.log 2>&1 || { tail -30 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
timeout -k 10 120 python tools/xt_phases.py run pair graph core save > $OUT/xt.txt 2>&1 || { tail -20 $OUT/xt.txt; exit 1; }
grep -v amdgpu $OUT/xt.txt
timeout -k 10 120 python tools/bench_head.py > $OUT/bh.txt 2>&1 || { tail -20 $OUT/bh.txt; exit 1; }
cat $OUT/bh.txt
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o head -- python tools/bench_head.py --iters 50 --fused-only 1 > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
python tools/kstats.py $OUT/prof/head_kernel_stats.csv 58 24
