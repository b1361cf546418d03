#!/bin/bash
# Serialized trunk kernel trace (tools/trunk_serial.py under rocprofv3) -> per-conv roofline table.
#   bash tools/gpu_trunk_serial.sh TAG
TAG=${1:-trunk}
R=$PWD
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python $R/tools/trunk_serial.py 8 > $OUT/trunk_serial.log 2>&1
rc=$?; echo "== trunk_serial rc=$rc"; tail -3 $OUT/trunk_serial.log
[ $rc -ne 0 ] && exit $rc
cd $R
f=$(find $OUT/prof -name '*kernel_trace.csv' | head -1)
python tools/trunk_table.py $f 8 > $OUT/trunk_table_serial.txt && tail -30 $OUT/trunk_table_serial.txt
echo SESSION_DONE
