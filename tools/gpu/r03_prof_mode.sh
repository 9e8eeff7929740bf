#!/bin/bash
# kernel-trace stats + stream breakdown of the bench command in one precision mode
# usage: r03_prof_mode.sh <tag> <dtype>
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r03_x6prof}
DT=${2:-bf16x6}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --dtype $DT --steps 10 --warmup 3 --no-cpu-baseline --no-fp32 > gpurun_out/${TAG}_prof.log 2>&1 || { tail -20 gpurun_out/${TAG}_prof.log; exit 1; }
grep '^{' gpurun_out/${TAG}_prof.log | cut -c1-400
python3 tools/prof_summary.py gpurun_out/${TAG}_prof/run_results.db > gpurun_out/${TAG}_kernel_stats.txt 2>&1 || true
python3 tools/stream_breakdown.py gpurun_out/${TAG}_prof/run_results.db > gpurun_out/${TAG}_streams.txt 2>&1 || true
rm -rf gpurun_out/${TAG}_prof
head -40 gpurun_out/${TAG}_kernel_stats.txt | cut -c1-100,110-175
head -12 gpurun_out/${TAG}_streams.txt
