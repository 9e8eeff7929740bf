#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/dpre_bitwise.py celeba 32 SVAE_WH2_NSW=2 2>&1 | grep -v amdgpu.ids || exit 1
SVAE_WH2_NSW=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_wgrad_bf16_gpu.py tests/test_headline_gpu.py > gpurun_out/nsw_t.log 2>&1 || { tail -20 gpurun_out/nsw_t.log; exit 1; }
tail -1 gpurun_out/nsw_t.log
for r in 1 2; do for v in 1 2; do
  SVAE_WH2_NSW=$v timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-fp32 > gpurun_out/nsw_b$v.log 2>&1 || exit 1
  echo "NSW=$v $(tail -1 gpurun_out/nsw_b$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], r["avg_launch_us"], r["frac"], r["isolated"]["avg_launch_us"], r["isolated"]["frac"])')"
done; done
