#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/dpre_bitwise.py celeba 32 SVAE_ACT_F32 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 300 python tools/dpre_bitwise.py tiny 4 SVAE_ACT_F32 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 300 python tools/dpre_bitwise.py c_v2_diag_noise_abl 16 SVAE_ACT_F32 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 600 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread tests/test_headline_gpu.py tests/test_engine_gpu.py tests/test_wgrad_bf16_gpu.py tests/test_gather_bf16_gpu.py tests/test_fused_adam_gpu.py tests/test_chain_variants_gpu.py > gpurun_out/act_t.log 2>&1; rc=$?
grep -E "headline|passed|failed" gpurun_out/act_t.log | tail -3; [ $rc -ne 0 ] && { grep -E "Error|assert" gpurun_out/act_t.log | head; exit 1; }
for v in 1 0 1 0; do
  SVAE_ACT_F32=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fp32 > gpurun_out/act_b$v.log 2>&1 || exit 1
  echo "ACT_F32=$v $(tail -1 gpurun_out/act_b$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], d["elbo_per_img"], r["avg_launch_us"])')"
done
