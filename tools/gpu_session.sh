#!/bin/bash
# One GPU call: tests, micro-benchmarks, bench, optional profiles.  Stops at the first step that ends
# in a fault / abort / timeout (exit codes other than 0 and pytest's 1).
#   bash tools/gpu_session.sh TAG "tests/test_a.py tests/test_b.py" [bench] [gemm] [conv] [prof] [pmcg]
TAG=$1; shift
TESTS=$1; shift
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -3 $OUT/$name.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name"; exit $rc; fi
  return 0
}
if [ -n "$TESTS" ]; then run pytest 600 python -m pytest $TESTS -q -x; fi
for step in "$@"; do
  case $step in
    bench) run bench 300 python bench.py --no-cpu-baseline; tail -1 $OUT/bench.log ;;
    gemm) run bench_gemm 300 python tools/bench_gemm.py; cat $OUT/bench_gemm.log ;;
    conv) run bench_conv 300 python tools/bench_conv.py; cat $OUT/bench_conv.log ;;
    prof) (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python $OLDPWD/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/prof.log 2>&1); echo "== prof rc=$?" ;;
    pmcg) bash tools/pmc_gemm.sh $TAG/pmcg ;;
    pmc) bash tools/gpu_pmc.sh $TAG/pmc ;;
    tprof) run torch_prof 300 python tools/torch_prof.py; cat $OUT/torch_prof.log ;;
  esac
done
echo SESSION_DONE
