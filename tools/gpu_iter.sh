#!/bin/bash
# Iteration session: selected GPU tests (TESTS), optional tool commands (TOOLS, ';'-separated), the bench line.
#   TESTS="tests/test_resnet_gpu.py -k halo" TOOLS="python tools/bench_conv.py --layers=layer1" bash tools/gpu_iter.sh TAG
TAG=${1:-iter}
R=$PWD
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
run() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -v amdgpu.ids $OUT/$name.log | tail -${TAILN:-6} | cut -c1-400
  if [ $rc -ne 0 ]; then echo "STOP after $name"; exit $rc; fi
  return 0
}
if [ -n "$TESTS" ]; then run pytest 600 python -u -m pytest $TESTS -x -q --timeout 200 --timeout-method thread; fi
i=0
IFS=';' read -ra CMDS <<< "$TOOLS"
for c in "${CMDS[@]}"; do
  [ -z "$c" ] && continue
  i=$((i+1)); TAILN=30 run tool$i 300 bash -c "$c"
done
if [ "${BENCH:-1}" = 1 ]; then run bench 400 python -u bench.py --no-cpu-baseline; fi
echo SESSION_DONE
