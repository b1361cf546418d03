#!/bin/bash
# Round-2 session m: WavLM attention waves-per-block A/B (tests + benches).
TAG=${1:-r2m}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
run() {
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -v amdgpu.ids $OUT/$name.log | tail -${TAILN:-3} | cut -c1-300
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name"; exit $rc; fi
  return 0
}
for NW in 5 10; do
  run wavlm_nw$NW 300 env MER_ATTN_NW=$NW python -u -m pytest tests/test_wavlm_gpu.py tests/test_wavlm_train_gpu.py -x -q --timeout 120 --timeout-method thread
done
for NW in 4 5 10 4; do
  run bench_nw$NW 200 env MER_ATTN_NW=$NW python -u bench.py --no-cpu-baseline --probe-steps 0 --probe-launches 0
done
echo SESSION_DONE
