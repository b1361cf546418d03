#!/bin/bash
# Head iteration: parity tests, standalone timing at two weight-gradient row splits, PMC HBM traffic passes.
TAG=${1:-head2}
R=$PWD
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_xattn_fused_gpu.py tests/test_head_gpu.py tests/test_graphs_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -20 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for rows in 256 512 128; do
  MER_XH_WGRAD_ROWS=$rows timeout -k 10 200 python -u tools/bench_head.py > $OUT/head_$rows.log 2>&1 || { tail $OUT/head_$rows.log; exit 1; }
  echo "rows $rows: $(grep fused $OUT/head_$rows.log)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python $R/tools/bench_head.py --iters 50 > $OUT/prof.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc/fetch -o run -- python $R/tools/pmc_head.py run > $OUT/pmc_fetch.log 2>&1 || { echo "pmc fetch failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc/write -o run -- python $R/tools/pmc_head.py run > $OUT/pmc_write.log 2>&1 || { echo "pmc write failed"; exit 1; }
cd $R && python tools/pmc_head.py summarize $OUT/pmc > $OUT/pmc_head.json && python -c "
import json; d=json.load(open('$OUT/pmc_head.json')); print('traffic/step', d.get('traffic_bytes_per_step')); [print(k, v) for k, v in (d.get('per_kernel') or {}).items()]"
python tools/kstats.py $OUT/prof/run_kernel_stats.csv 1 40 | grep -E "xh_|total"
