#!/bin/bash
# Round-2 session k: stage-2 dropout tests, wgrad split sweep, full GPU suite, benches.
TAG=${1:-r2k}
bash tools/gpu_r2j.sh $TAG || exit $?
bash tools/gpu_r2i.sh $TAG/sweep || exit $?
echo ALL_DONE
