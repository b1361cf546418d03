#!/bin/bash
# Board power / clocks while the default bench runs (is the train step at the power cap?).
#   bash tools/power_probe.sh TAG
TAG=${1:-power}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
rocm-smi --showpower --showclocks --showmaxpower > $OUT/idle.txt 2>&1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 8000 --warmup 10 > $OUT/bench.log 2>&1 &
BP=$!
for i in $(seq 1 20); do sleep 2; rocm-smi --showpower --showclocks > $OUT/busy_$i.txt 2>&1; done
wait $BP
echo "bench rc=$?"
grep -E "Power|sclk|Max" $OUT/idle.txt | head -8
for i in $(seq 1 20); do echo "t=$((2*i))s $(grep -E "Package Power|sclk clock level" $OUT/busy_$i.txt | tr -s " " | tr "\n" " ")"; done
grep '^{' $OUT/bench.log | cut -c1-200
