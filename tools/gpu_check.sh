#!/bin/bash
# Quick GPU session: the GPU suite, smoke, the default bench line and (with C5=1) the C5 inference line.
#   bash tools/gpu_check.sh TAG
TAG=${1:-check}
R=$PWD
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
run() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -v amdgpu.ids $OUT/$name.log | tail -${TAILN:-4} | cut -c1-600
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name"; exit $rc; fi
  return 0
}
run pytest 900 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread
run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')"
run bench 600 python -u bench.py
if [ "${C5:-0}" = 1 ]; then run bench_c5 600 python -u bench.py --c5 --steps 20 --warmup 5; fi
echo SESSION_DONE
