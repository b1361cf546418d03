#!/bin/bash
# 128x128 tiles for WavLM conv2/conv3: full GPU suite, smoke, bench (x2).
R=$PWD; OUT=$R/gpurun_out/r2za; mkdir -p $OUT
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > $OUT/smoke.log 2>&1; rc=$?; tail -1 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --probe-steps 0 > $OUT/bench_$i.log 2>&1; rc=$?; tail -1 $OUT/bench_$i.log | cut -c100-200; [ $rc -eq 0 ] || exit $rc
done
