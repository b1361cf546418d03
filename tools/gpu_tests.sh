#!/bin/bash
# GPU test pass: the given test files first (verbose), then optionally the whole -m gpu suite.
# Usage: bash tools/gpu_tests.sh TAG "tests/a.py tests/b.py" [--all]
TAG=${1:-run}
FILES=$2
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
rc=0
if [ -n "$FILES" ]; then
  timeout -k 10 900 python -u -m pytest $FILES -m gpu -v --timeout 600 --timeout-method thread -s > $OUT/focus.log 2>&1
  rc=$?
  echo "FOCUS_EXIT $rc" >> $OUT/focus.log
  grep -E "PASSED|FAILED|ERROR|passed|failed" $OUT/focus.log | tail -30
fi
if [ "$3" == "--all" ] && { [ $rc -eq 0 ] || [ $rc -eq 1 ]; }; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/all.log 2>&1
  echo "ALL_EXIT $?" >> $OUT/all.log
  tail -15 $OUT/all.log
fi
