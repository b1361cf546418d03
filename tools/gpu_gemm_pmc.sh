#!/bin/bash
# conv1 GEMM in isolation: timing of the given variants + FETCH_SIZE / WRITE_SIZE passes.  Usage: TAG [variants]
TAG=${1:-gemm}
V=${2:-13}
R=$PWD
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -u tools/bench_gemm.py --shapes=conv1,conv2,qkv,ffn1 --variants=$V > $OUT/gemm.log 2>&1 || { tail $OUT/gemm.log; exit 1; }
grep TF/s $OUT/gemm.log
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc/fetch -o run -- python $R/tools/bench_gemm.py --shapes=conv1 --variants=18 > $OUT/pmc_fetch.log 2>&1 || { echo "pmc fetch failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc/write -o run -- python $R/tools/bench_gemm.py --shapes=conv1 --variants=18 > $OUT/pmc_write.log 2>&1 || { echo "pmc write failed"; exit 1; }
cd $R && python tools/pmc_traffic.py $OUT/pmc
