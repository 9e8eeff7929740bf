#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python tools/bench_wgrad.py 20 2 step 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/wgiso_prof -o run -- python3 tools/bench_wgrad.py 20 2 step > gpurun_out/wgiso_prof.log 2>&1 || exit 1
python3 tools/prof_summary.py gpurun_out/wgiso_prof/run_results.db > gpurun_out/wgiso_kernel_stats.txt 2>&1 || true
head -16 gpurun_out/wgiso_kernel_stats.txt | cut -c1-70,110-175
