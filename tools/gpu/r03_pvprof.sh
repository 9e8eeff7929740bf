#!/bin/bash
# c_pixelvae bench leg under the kernel-trace profiler: per-kernel stats of the head at B = 128
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r03_pv}
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --config c_pixelvae --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_prof.log 2>&1 || { tail -20 gpurun_out/${TAG}_prof.log; exit 1; }
tail -1 gpurun_out/${TAG}_prof.log | cut -c1-300
python3 tools/prof_summary.py gpurun_out/${TAG}_prof/run_results.db > gpurun_out/${TAG}_kernel_stats.txt 2>&1 || true
rm -rf gpurun_out/${TAG}_prof
head -40 gpurun_out/${TAG}_kernel_stats.txt | cut -c1-160
