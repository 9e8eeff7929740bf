#!/bin/bash
# stride-1 weight-GEMM prefetch depth (SVAE_WH2_PF 1 vs 2): parity, isolated shapes, step
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_wgrad_bf16_gpu.py tests/test_halo_gpu.py tests/test_headline_gpu.py > gpurun_out/pf_t.log 2>&1 || { tail -30 gpurun_out/pf_t.log; exit 1; }
tail -1 gpurun_out/pf_t.log
for pf in 1 2; do
  SVAE_WH2_PF=$pf timeout -k 10 300 python tools/bench_wgrad.py 20 2 step > gpurun_out/pf_w$pf.log 2>&1 || { tail -5 gpurun_out/pf_w$pf.log; exit 1; }
  echo "PF=$pf"; grep -E "dec s1|enc b|inf b|total" gpurun_out/pf_w$pf.log
done
for r in 1 2; do for pf in 1 2; do
  SVAE_WH2_PF=$pf timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-fp32 > gpurun_out/pf_b.log 2>&1 || exit 1
  echo "PF=$pf $(tail -1 gpurun_out/pf_b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], d["elbo_per_img"], r["avg_launch_us"], r["frac"], r["isolated"]["avg_launch_us"])')"
done; done
