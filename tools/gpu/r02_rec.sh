#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
SVAE_REC_GROUP=2 timeout -k 10 500 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread tests/test_engine_gpu.py tests/test_headline_gpu.py tests/test_fused_adam_gpu.py tests/test_dp_overlap_gpu.py > gpurun_out/rec_t.log 2>&1; rc=$?
grep -E "headline|passed|failed" gpurun_out/rec_t.log | tail -4; [ $rc -ne 0 ] && { grep -E "Error|assert" gpurun_out/rec_t.log | head; exit 1; }
for v in 0 1 2 4 0 1 2; do
  SVAE_REC_GROUP=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fp32 > gpurun_out/rec_b$v.log 2>&1 || exit 1
  echo "REC_GROUP=$v $(tail -1 gpurun_out/rec_b$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["elbo_per_img"])')"
done
