#!/bin/bash
# profile + bench only
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bf16 -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/prof.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench.log 2>&1 || exit 1
