#!/bin/bash
# One full GPU call: GPU parity tests, the default bench line (with cpu_baseline), a kernel-trace
# profile of the bench, and the PMC HBM-traffic passes for the probe kernel.  Stops at the first step
# that faults / aborts / times out.   Usage: bash tools/gpu_full.sh TAG [notests|tests] [nopmc]
TAG=${1:-full}
R=$PWD
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
stop() { echo "STOP after $1 (rc=$2)"; exit $2; }
if [ "$2" != "notests" ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
  rc=$?; echo "== pytest rc=$rc"; tail -4 $OUT/pytest_gpu.log
  [ $rc -ne 0 ] && stop pytest $rc
fi
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1
rc=$?; echo "== bench rc=$rc"; tail -1 $OUT/bench.log
[ $rc -ne 0 ] && { tail -20 $OUT/bench.log; stop bench $rc; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/prof.log 2>&1
rc=$?; echo "== prof rc=$rc"; [ $rc -ne 0 ] && stop prof $rc
[ "$3" == "nopmc" ] && { echo SESSION_DONE; exit 0; }
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc/fetch -o run -- python $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/pmc_fetch.log 2>&1
rc=$?; echo "== pmc fetch rc=$rc"; [ $rc -ne 0 ] && stop pmc_fetch $rc
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc/write -o run -- python $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/pmc_write.log 2>&1
rc=$?; echo "== pmc write rc=$rc"; [ $rc -ne 0 ] && stop pmc_write $rc
echo SESSION_DONE
