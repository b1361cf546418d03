#!/bin/bash
# conv0 moment statistics: WavLM GPU tests first, then the full suite, bench line, kernel-trace stats.
R=$PWD; OUT=$R/gpurun_out/r2v; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_wavlm_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest_wavlm.log 2>&1; rc=$?; tail -15 $OUT/pytest_wavlm.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -15 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench.log 2>&1; rc=$?; tail -1 $OUT/bench.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python $R/bench.py --steps 20 --warmup 5 --probe-steps 5 --no-cpu-baseline > $OUT/prof.log 2>&1; echo "prof rc=$?"
