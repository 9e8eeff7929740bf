#!/bin/bash
# kernel-trace stats + stream breakdown of the bench command, and the weight-GEMMs timed alone
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r02_v40}
timeout -k 10 200 python tools/bench_wgrad.py 20 2 step > gpurun_out/${TAG}_wgrad_isolated.txt 2>&1 || { tail gpurun_out/${TAG}_wgrad_isolated.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/${TAG}_wgrad_isolated.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-fp32 > gpurun_out/${TAG}_prof.log 2>&1 || exit 1
python3 tools/prof_summary.py gpurun_out/${TAG}_prof/run_results.db > gpurun_out/${TAG}_kernel_stats.txt 2>&1 || true
python3 tools/stream_breakdown.py gpurun_out/${TAG}_prof/run_results.db 28 20 8 > gpurun_out/${TAG}_streams.txt 2>&1 || true
head -45 gpurun_out/${TAG}_streams.txt
