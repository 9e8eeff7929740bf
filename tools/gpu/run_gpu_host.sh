#!/bin/bash
# host enqueue rate vs GPU rate (side stream on / off)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/host_rate.py > gpurun_out/host.log 2>&1 || exit 1
SVAE_NO_SIDE=1 timeout -k 10 300 python tools/host_rate.py > gpurun_out/host_noside.log 2>&1 || exit 1
