#!/bin/bash
# wave-split small-image gather: parity (op + engine bf16) then microbench / bench A/B
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gather_bf16_gpu.py -k "path2 or 2-" > gpurun_out/kw_t1.log 2>&1; rc=$?
tail -3 gpurun_out/kw_t1.log; [ $rc -ne 0 ] && { grep -E "Error|assert" gpurun_out/kw_t1.log | head -20; exit 1; }
timeout -k 10 500 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread tests/test_headline_gpu.py tests/test_engine_gpu.py -k "bf16 or headline" > gpurun_out/kw_t2.log 2>&1; rc=$?
grep -E "headline|bf16 [0-9]|loss rel|passed|failed" gpurun_out/kw_t2.log | tail -12; [ $rc -ne 0 ] && exit 1
SVAE_NO_KW=1 timeout -k 10 120 python tools/bench_gather.py 2 > gpurun_out/kw_mb0.log 2>&1 && timeout -k 10 120 python tools/bench_gather.py 2 > gpurun_out/kw_mb1.log 2>&1 || exit 1
paste gpurun_out/kw_mb0.log gpurun_out/kw_mb1.log | cut -c1-150
for v in 1 0 1 0; do
  SVAE_NO_KW=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fp32 > gpurun_out/kw_b$v.log 2>&1 || exit 1
  echo "NO_KW=$v $(tail -1 gpurun_out/kw_b$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["elbo_per_img"])')"
done
