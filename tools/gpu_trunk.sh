#!/bin/bash
# trunk-focused pass: ResNet / e2e GPU tests, bench line, kernel trace -> per-layer trunk table.  Usage: TAG
TAG=${1:-trunk}
R=$PWD
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
bash tools/gpu_tests.sh $TAG "tests/test_resnet_gpu.py tests/test_e2e_gpu.py tests/test_e2e_c2_gpu.py" || exit 1
grep -E "passed|failed" $OUT/focus.log | tail -1
timeout -k 10 400 python -u bench.py --no-cpu-baseline --probe-steps 0 > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o run -- python $R/bench.py --steps 8 --warmup 3 --probe-steps 0 --no-cpu-baseline > $OUT/prof.log 2>&1
echo "PROF_EXIT $?"
cd $R && python tools/trunk_table.py $OUT/prof/run_kernel_trace.csv 11 > $OUT/trunk_table.txt 2>&1; grep "#" $OUT/trunk_table.txt | head -20
