#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu/r02_gap.sh ${1:-r02_gap2} || exit 1
timeout -k 10 300 python tools/bench_pcnn.py --batch 16 > gpurun_out/pcnn_b16.log 2>&1 || { tail -20 gpurun_out/pcnn_b16.log; exit 1; }
tail -1 gpurun_out/pcnn_b16.log
