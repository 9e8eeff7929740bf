#!/bin/bash
# parity subset, per-layer GEMM trace, then two bench runs
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_headline_gpu.py tests/test_engine_gpu.py tests/test_pcnn_gpu.py > gpurun_out/t2_t.log 2>&1 || { tail -30 gpurun_out/t2_t.log; exit 1; }
tail -1 gpurun_out/t2_t.log
SVAE_TRACE_GEMM=1 timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-fp32 > gpurun_out/trace.log 2> gpurun_out/trace.err || { tail -20 gpurun_out/trace.err; exit 1; }
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-fp32 > gpurun_out/t2_b.log 2>&1 || exit 1
  echo "bench $(tail -1 gpurun_out/t2_b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["elbo_per_img"])')"
done
