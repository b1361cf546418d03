#!/bin/bash
# s2d-into-static-input check: full GPU suite, smoke, bench line, kernel-trace stats of the bench command.
R=$PWD; OUT=$R/gpurun_out/r2u; mkdir -p $OUT
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > $OUT/smoke.log 2>&1; rc=$?; tail -1 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench.log 2>&1; rc=$?; tail -1 $OUT/bench.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python $R/bench.py --steps 20 --warmup 5 --probe-steps 5 --no-cpu-baseline > $OUT/prof.log 2>&1; echo "prof rc=$?"
