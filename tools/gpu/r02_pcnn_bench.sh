#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/bench_pcnn.py --batch 16 --cpu > gpurun_out/pcnn_b16.log 2>&1 || { tail -20 gpurun_out/pcnn_b16.log; exit 1; }
tail -1 gpurun_out/pcnn_b16.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pcnn_prof -o run -- python3 tools/bench_pcnn.py --batch 16 --steps 3 --warmup 1 > gpurun_out/pcnn_prof.log 2>&1 || exit 1
python3 tools/prof_summary.py gpurun_out/pcnn_prof/run_results.db > gpurun_out/pcnn_kernel_stats.txt 2>&1 || true
head -25 gpurun_out/pcnn_kernel_stats.txt | cut -c1-60,110-175
