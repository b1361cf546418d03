#!/bin/bash
# Kernel trace of the default train step (bench.py under rocprofv3) -> per-kernel summary per step.
#   bash tools/gpu_step_prof.sh TAG
TAG=${1:-stepprof}
R=$PWD
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python $R/bench.py --steps 20 --warmup 5 --probe-steps 0 --probe-launches 0 --no-cpu-baseline > $OUT/prof.log 2>&1
rc=$?; echo "== prof rc=$rc"; grep '^{' $OUT/prof.log | cut -c1-200
[ $rc -ne 0 ] && { tail -20 $OUT/prof.log; exit $rc; }
cd $R
python tools/kstats.py $(find $OUT/prof -name '*kernel_stats.csv' | head -1) 25 40 > $OUT/kstats.txt
cat $OUT/kstats.txt
