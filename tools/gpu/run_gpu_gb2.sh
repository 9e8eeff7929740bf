#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/bench_gather.py 0 > gpurun_out/gb_p0.log 2>&1 || exit 1
SVAE_HALO_ALL=1 timeout -k 10 300 python tools/bench_gather.py 1 > gpurun_out/gb_p1.log 2>&1 || exit 1
