#!/bin/bash
# bench line + steady-state kernel trace.  Usage: bash tools/gpu_prof.sh TAG [bench args...]
TAG=${1:-prof}
shift
R=$PWD
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u bench.py --no-cpu-baseline "$@" > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python $R/bench.py --steps 8 --warmup 3 --probe-steps 0 --no-cpu-baseline "$@" > $OUT/prof.log 2>&1
echo "PROF_EXIT $?"
cd $R
python tools/kstats_trace.py $(ls $OUT/prof/*kernel_trace.csv | head -1) 45 > $OUT/steady.txt 2>&1
head -50 $OUT/steady.txt
