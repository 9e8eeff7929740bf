#!/bin/bash
# kernel-trace stats of the bench command + stream breakdown
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r02_v3}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-fp32 > gpurun_out/${TAG}_prof.log 2>&1 || exit 1
python3 tools/prof_summary.py gpurun_out/${TAG}_prof/run_results.db > gpurun_out/${TAG}_kernel_stats.txt 2>&1 || true
head -40 gpurun_out/${TAG}_kernel_stats.txt
python3 tools/stream_breakdown.py gpurun_out/${TAG}_prof/run_results.db > gpurun_out/${TAG}_streams.txt 2>&1 || true
cat gpurun_out/${TAG}_streams.txt | head -30
