#!/bin/bash
# PMC passes over tools/bench_gemm.py (one counter group per pass).  Usage: bash tools/pmc_gemm.sh TAG
TAG=${1:-pmcg}
R=$PWD
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- python $R/tools/bench_gemm.py --quick > $OUT/p$i.log 2>&1 || { echo "pass $i ($grp) failed"; tail -5 $OUT/p$i.log; exit 1; }
done
echo PMC_OK
