#!/bin/bash
# Round-2 session h: GEMM tile-order A/B (time + HBM traffic of conv1), WavLM test.
TAG=${1:-r2h}
R=$PWD
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
run() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -v amdgpu.ids $OUT/$name.log | tail -${TAILN:-12} | cut -c1-300
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name"; exit $rc; fi
  return 0
}
run wavlm 300 python -u -m pytest tests/test_wavlm_gpu.py -x -q --timeout 120 --timeout-method thread
run gemm_g8 200 env MER_GEMM_GROUP=8 python -u tools/bench_gemm.py --shapes=conv1,conv2 --variants=13
run gemm_g1 200 python -u tools/bench_gemm.py --shapes=conv1,conv2 --variants=13
cd /tmp && export TMPDIR=/tmp
for G in 8 1; do
  MER_GEMM_GROUP=$G timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_g$G/fetch -o run -- python $R/tools/bench_gemm.py --shapes=conv1 --variants=13 > $OUT/pmc_fetch_g$G.log 2>&1 || { echo "pmc fetch failed"; exit 1; }
  MER_GEMM_GROUP=$G timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_g$G/write -o run -- python $R/tools/bench_gemm.py --shapes=conv1 --variants=13 > $OUT/pmc_write_g$G.log 2>&1 || { echo "pmc write failed"; exit 1; }
  (cd $R && python tools/pmc_traffic.py $OUT/pmc_g$G)
done
echo SESSION_DONE
