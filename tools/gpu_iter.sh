#!/bin/bash
# One build -> measure iteration on the GPU box: focused tests, then the default bench line (no CPU baseline).
#   bash tools/gpu_iter.sh TAG "tests/a.py tests/b.py" [extra bench args]
TAG=${1:-iter}
FILES=$2
shift 2
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
if [ -n "$FILES" ]; then
  timeout -k 10 600 python -u -m pytest $FILES -m gpu -q -x --timeout 200 --timeout-method thread > $OUT/focus.log 2>&1
  rc=$?
  tail -5 $OUT/focus.log
  if [ $rc -ne 0 ]; then echo "FOCUS_EXIT $rc"; exit $rc; fi
fi
timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > $OUT/bench.log 2>&1
rc=$?
grep '^{' $OUT/bench.log | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); h=d.get('roofline_head') or {}
    print('BENCH', d['value'], d['ms_per_step'], d.get('ms_per_step_median'), 'head', {k: h.get(k) for k in ('frac','fwd_ms','bwd_ms','ms_per_step')}, 'core', (h.get('core') or {}).get('kernel_ms'), (h.get('core') or {}).get('frac'))"
exit $rc
