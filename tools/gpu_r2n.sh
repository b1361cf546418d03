#!/bin/bash
# Round-2 session n: every GEMM variant on the WavLM encoder shapes (production epilogues).
TAG=${1:-r2n}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -u tools/bench_gemm.py --shapes=out_proj,ffn2 --variants=9,1,2,3,4,5,6,7,8,10,11,12,13 --resid32 > $OUT/resid.log 2>&1 || exit $?
grep TF/s $OUT/resid.log
timeout -k 10 300 python -u tools/bench_gemm.py --shapes=qkv,ffn1 --variants=13,1,2,3,4,5,6,7,8,9,10,11,12 > $OUT/plain.log 2>&1 || exit $?
grep TF/s $OUT/plain.log
echo SESSION_DONE
