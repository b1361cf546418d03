#!/bin/bash
# conv0 moments A/B: the WavLM tail oracle test's noisiest gradient under the previous build, and the bench line
# under both builds on the same box.
R=$PWD; OUT=$R/gpurun_out/r2x; mkdir -p $OUT
MER_HIP_LIB=$R/tools/_ab/libOld.so timeout -k 10 300 python -u -m pytest tests/test_wavlm_stage2_gpu.py -x -q -s --timeout 200 --timeout-method thread -k "tail_forward_backward_vs_oracle" > $OUT/tail_old.log 2>&1; rc=$?
echo "== tail old rc=$rc"; grep "gru_rel_pos_linear.bias" $OUT/tail_old.log; [ $rc -le 1 ] || exit $rc
for v in Old Cur Old Cur; do
  if [ $v = Cur ]; then L=$R/multimodalemotionrecognition_amd/libmer_hip.so; else L=$R/tools/_ab/lib$v.so; fi
  MER_HIP_LIB=$L timeout -k 10 300 python -u bench.py --no-cpu-baseline --probe-steps 0 > $OUT/bench_$v.log 2>&1; rc=$?
  echo "== bench $v rc=$rc"; tail -1 $OUT/bench_$v.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
done
