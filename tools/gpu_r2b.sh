#!/bin/bash
# round-2 session b: new WavLM train-mode tests + re-run of the failures, full suite, then a bench line
OUT=$PWD/gpurun_out/r2b
mkdir -p $OUT
bash tools/gpu_tests.sh r2b "tests/test_wavlm_train_gpu.py tests/test_round2_features_gpu.py tests/test_e2e_c2_gpu.py tests/test_e2e_gpu.py" --all
timeout -k 10 600 python -u bench.py --no-cpu-baseline > $OUT/bench.log 2>&1
echo "BENCH_EXIT $?"
tail -2 $OUT/bench.log
