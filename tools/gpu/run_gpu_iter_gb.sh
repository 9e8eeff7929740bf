#!/bin/bash
# iteration + image-space gather microbench
cd $GRAFT_REPO_ROOT
bash tools/gpu/run_gpu_iter.sh || exit 1
timeout -k 10 300 python tools/bench_gather.py image 1 2 > gpurun_out/gb.log 2>&1 || exit 1
