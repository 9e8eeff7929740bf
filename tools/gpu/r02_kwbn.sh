#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
SVAE_KW_BN=64 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gather_bf16_gpu.py -k "2-" > gpurun_out/kwbn_t1.log 2>&1; rc=$?
tail -2 gpurun_out/kwbn_t1.log; [ $rc -ne 0 ] && { grep -E "Error|assert" gpurun_out/kwbn_t1.log | head -20; exit 1; }
SVAE_KW_BN=32 timeout -k 10 120 python tools/bench_gather.py 2 > gpurun_out/kwbn_mb32.log 2>&1 && SVAE_KW_BN=64 timeout -k 10 120 python tools/bench_gather.py 2 > gpurun_out/kwbn_mb64.log 2>&1 || exit 1
paste gpurun_out/kwbn_mb32.log gpurun_out/kwbn_mb64.log | cut -c1-150
for v in 32 64 32 64; do
  SVAE_KW_BN=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fp32 > gpurun_out/kwbn_b$v.log 2>&1 || exit 1
  echo "KW_BN=$v $(tail -1 gpurun_out/kwbn_b$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["elbo_per_img"])')"
done
