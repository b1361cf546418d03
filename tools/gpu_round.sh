#!/bin/bash
# One GPU session: tests, bench, kernel-trace profile.  Usage: bash tools/gpu_round.sh TAG [--no-tests]
TAG=${1:-run}
R=$PWD
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
if [ "$2" != "--no-tests" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q -x > $OUT/pytest_gpu.log 2>&1
  echo "PYTEST_EXIT $?" >> $OUT/pytest_gpu.log
  tail -3 $OUT/pytest_gpu.log
fi
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/prof.log 2>&1
echo "PROF_EXIT $?"
