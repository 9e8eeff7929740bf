#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_dp_overlap_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/dp.log 2>&1
echo rc=$? >> gpurun_out/dp.log
