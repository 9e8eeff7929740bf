#!/bin/bash
# parity subset + bench + kernel-trace stream/gap breakdown
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r02_gap}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_headline_gpu.py tests/test_engine_gpu.py tests/test_chain_variants_gpu.py tests/test_fused_adam_gpu.py > gpurun_out/${TAG}_t.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/${TAG}_t.log | tail -2; [ $rc -ne 0 ] && { grep -E "Error|assert" gpurun_out/${TAG}_t.log | head; exit 1; }
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fp32 > gpurun_out/${TAG}_b$i.log 2>&1 || exit 1
  echo "bench $(tail -1 gpurun_out/${TAG}_b$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], d["elbo_per_img"], r["avg_launch_us"])')"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-fp32 > gpurun_out/${TAG}_prof.log 2>&1 || exit 1
python3 tools/prof_summary.py gpurun_out/${TAG}_prof/run_results.db > gpurun_out/${TAG}_kernel_stats.txt 2>&1 || true
python3 tools/stream_breakdown.py gpurun_out/${TAG}_prof/run_results.db 8 12 > gpurun_out/${TAG}_streams.txt 2>&1 || true
grep -A 30 "main stream" gpurun_out/${TAG}_streams.txt
