#!/bin/bash
# Same-box A/B of the working tree against an older build tree (tools/scratch/abtree: `git archive <rev>` +
# its own in-tree libraries), alternating default bench runs.
#   bash tools/gpu_ab_tree.sh TAG [rounds] [env for the old tree]
TAG=${1:-abtree}; N=${2:-2}; OLDENV=${3:-}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
R=$PWD
run_new() {
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --probe-launches 0 --probe-steps 0 > $OUT/new_$1.log 2>&1 || { echo "FAIL new"; tail -5 $OUT/new_$1.log; exit 1; }
  echo "new run $1: $(grep '^{' $OUT/new_$1.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["ms_per_step_median"])')"
}
run_old() {
  (cd tools/scratch/abtree && env $OLDENV timeout -k 10 300 python -u bench.py --no-cpu-baseline --probe-launches 0 --probe-steps 0) > $OUT/old_$1.log 2>&1 || { echo "FAIL old"; tail -5 $OUT/old_$1.log; exit 1; }
  echo "old run $1: $(grep '^{' $OUT/old_$1.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["ms_per_step_median"])')"
}
# ABBA order: odd rounds run the working tree first, even rounds the old tree first
for i in $(seq 1 $N); do
  if [ $((i % 2)) = 1 ]; then run_new $i; run_old $i; else run_old $i; run_new $i; fi
done
