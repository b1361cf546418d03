#!/bin/bash
# Round-end measurement session: GPU suite, smoke, the default bench line (with the CPU baseline), a kernel-trace
# profile of the same bench command, and the conv1 HBM-traffic PMC passes (separate --pmc runs).
#   bash tools/gpu_final.sh TAG
TAG=${1:-final}
R=$PWD
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
run() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -v amdgpu.ids $OUT/$name.log | tail -${TAILN:-4} | cut -c1-400
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name"; exit $rc; fi
  return 0
}
run pytest 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread
run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')"
run bench 600 python -u bench.py
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python $R/bench.py --steps 20 --warmup 5 --probe-steps 5 --no-cpu-baseline > $OUT/prof.log 2>&1
echo "== prof rc=$?"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc/fetch -o run -- python $R/tools/bench_gemm.py --shapes=conv1 --variants=23 --gelu > $OUT/pmc_fetch.log 2>&1 || { echo "pmc fetch failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc/write -o run -- python $R/tools/bench_gemm.py --shapes=conv1 --variants=23 --gelu > $OUT/pmc_write.log 2>&1 || { echo "pmc write failed"; exit 1; }
cd $R && python tools/pmc_traffic.py $OUT/pmc > $OUT/pmc_traffic.json && cat $OUT/pmc_traffic.json
cd /tmp
# the fused head's HBM traffic and MFMA busy fraction (tools/pmc_head.py): one counter group per pass
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmch/fetch -o run -- python $R/tools/pmc_head.py run > $OUT/pmch_fetch.log 2>&1 || { echo "head pmc fetch failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmch/write -o run -- python $R/tools/pmc_head.py run > $OUT/pmch_write.log 2>&1 || { echo "head pmc write failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmch/mfma -o run -- python $R/tools/pmc_head.py run > $OUT/pmch_mfma.log 2>&1 || { echo "head pmc mfma failed"; exit 1; }
cd $R && python tools/pmc_head.py summarize $OUT/pmch > $OUT/pmc_traffic_head.json && grep traffic_bytes $OUT/pmc_traffic_head.json
# the serialized per-conv roofline table of the same tree
bash tools/gpu_trunk_serial.sh ${TAG}_trunk > $OUT/trunk.log 2>&1 && grep "^# " $R/gpurun_out/${TAG}_trunk/trunk_table_serial.txt | head -4
echo SESSION_DONE
