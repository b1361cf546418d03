#!/bin/bash
# Kernel traces of single-mode C4 sweep runs (one rocprofv3 pass per mode).
TAG=${1:-sweepprof}
R=$PWD
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for m in concat xattn; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$m -o run -- python $R/tools/bench_sweep.py --modes $m --steps 20 --warmup 10 > $OUT/$m.log 2>&1 || exit 1
  grep '^{' $OUT/$m.log
done
cd $R
for m in concat xattn; do echo "== $m"; python tools/kstats.py $OUT/$m/run_kernel_stats.csv 30 25 | cut -c1-150; done
