#!/bin/bash
# A/B of the conv0 statistics on the end-to-end oracle step: previous build, moments + rounded input, current.
R=$PWD; OUT=$R/gpurun_out/r2w; mkdir -p $OUT
for v in Old R Cur; do
  if [ $v = Cur ]; then L=$R/multimodalemotionrecognition_amd/libmer_hip.so; else L=$R/tools/_ab/lib$v.so; fi
  MER_HIP_LIB=$L timeout -k 10 300 python -u -m pytest tests/test_e2e_gpu.py -x -q -s --timeout 200 --timeout-method thread -k "train_step_vs_oracle" > $OUT/e2e_$v.log 2>&1; rc=$?
  echo "== $v rc=$rc"; grep "loss hip" $OUT/e2e_$v.log
  [ $rc -le 1 ] || exit $rc
done
