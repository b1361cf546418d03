#!/bin/bash
# Same-box A/B of environment switches on the default bench (alternating runs, no CPU baseline).
#   bash tools/gpu_ab.sh TAG "ENV_A" "ENV_B" [rounds]
TAG=${1:-ab}; A=$2; B=$3; N=${4:-2}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
for i in $(seq 1 $N); do
  for cfg in "$A" "$B"; do
    name=$(echo "$cfg" | tr ' =/' '_-_')
    env $cfg timeout -k 10 300 python -u bench.py --no-cpu-baseline --probe-launches 0 --probe-steps 0 > $OUT/${name}_$i.log 2>&1 || { echo "FAIL $cfg"; tail -5 $OUT/${name}_$i.log; exit 1; }
    echo "$cfg run $i: $(grep '^{' $OUT/${name}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["ms_per_step_median"])')"
  done
done
