#!/bin/bash
# Round-2 session s: single-pass wgrad fold threshold A/B.
TAG=${1:-r2s}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
for F in 16 64 160; do
  MER_WGRAD_FOLD_MAX=$F timeout -k 10 200 python -u tools/bench_conv.py --variants= --wgrad-variants=4 > $OUT/fold$F.log 2>&1 || exit $?
  echo "== fold_max $F"; grep -v amdgpu.ids $OUT/fold$F.log | cut -c1-60
done
echo SESSION_DONE
