#!/bin/bash
# GPU suite, then a same-box ABBA of the default bench against the old tree in tools/scratch/abtree.
#   bash tools/gpu_suite_ab.sh TAG [rounds]
TAG=${1:-suite_ab}; N=${2:-2}
R=$PWD
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "== pytest rc=$rc"; tail -3 $OUT/pytest.log
[ $rc -ne 0 ] && exit $rc
bash tools/gpu_ab_tree.sh $TAG $N
