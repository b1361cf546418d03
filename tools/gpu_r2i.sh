#!/bin/bash
# Round-2 session i: wgrad split-count sweep (kernel + fold) on the pipelined variant.
TAG=${1:-r2i}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
for cfg in "768 0" "512 0" "768 2048" "512 2048" "384 4096" "256 4096"; do
  set -- $cfg
  MER_WGRAD_WGS=$1 MER_WGRAD_MIN_PIX=$2 timeout -k 10 200 python -u tools/bench_conv.py --variants= --wgrad-variants=4 > $OUT/w_$1_$2.log 2>&1
  rc=$?
  echo "== wgs=$1 minpix=$2 rc=$rc"; grep -v amdgpu.ids $OUT/w_$1_$2.log | cut -c1-60
  if [ $rc -ne 0 ]; then exit $rc; fi
done
echo SESSION_DONE
