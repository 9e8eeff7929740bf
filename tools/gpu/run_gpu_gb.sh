#!/bin/bash
# gather microbench (image-space shapes) + kernel trace of it
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/bench_gather.py image 0 1 2 > gpurun_out/gb.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gb -o run -- python3 tools/bench_gather.py image 0 1 2 > gpurun_out/gb_prof.log 2>&1 || exit 1
