#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gather_bf16_gpu.py > gpurun_out/kw2_t1.log 2>&1; rc=$?
tail -2 gpurun_out/kw2_t1.log; [ $rc -ne 0 ] && { grep -E "Error|assert" gpurun_out/kw2_t1.log | head -20; exit 1; }
timeout -k 10 500 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread tests/test_headline_gpu.py tests/test_engine_gpu.py tests/test_fused_adam_gpu.py -k "bf16 or headline" > gpurun_out/kw2_t2.log 2>&1; rc=$?
grep -E "headline|passed|failed" gpurun_out/kw2_t2.log | tail -4; [ $rc -ne 0 ] && exit 1
for v in 0 1 2 1 2; do
  SVAE_KW=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fp32 > gpurun_out/kw2_b$v.log 2>&1 || exit 1
  echo "KW=$v $(tail -1 gpurun_out/kw2_b$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["elbo_per_img"])')"
done
