#!/bin/bash
# Kernel traces of the bench step under three settings (prefetch off; graphs off; default) to find what
# serialises the main stream behind the side stream.  Usage: bash tools/gap_probe.sh TAG
R=$PWD; OUT=$R/gpurun_out/$1; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/nopf -o run -- python $R/bench.py --steps 6 --warmup 3 --no-cpu-baseline --no-prefetch > $OUT/nopf.log 2>&1 || exit 1
MER_GRAPHS=0 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/nograph -o run -- python $R/bench.py --steps 6 --warmup 3 --no-cpu-baseline > $OUT/nograph.log 2>&1 || exit 1
echo PROBE_DONE
