#!/bin/bash
# host enqueue cost vs GPU time per step (no profiler)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/host_enqueue.py 40 > gpurun_out/host2.txt 2>&1 || { tail -20 gpurun_out/host2.txt; exit 1; }
cat gpurun_out/host2.txt
