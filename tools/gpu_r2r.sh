#!/bin/bash
# Round-2 session r: 32-wide K deep-ring GEMM variants vs production picks (bit-identity via maxdiff, speed).
TAG=${1:-r2r}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -u tools/bench_gemm.py --shapes=conv1,conv2,qkv,ffn1 --variants=13,15 > $OUT/big.log 2>&1 || exit $?
grep TF/s $OUT/big.log
timeout -k 10 300 python -u tools/bench_gemm.py --shapes=ffn2,out_proj --variants=7,16,9,17 --resid32 > $OUT/resid.log 2>&1 || exit $?
grep TF/s $OUT/resid.log
echo SESSION_DONE
