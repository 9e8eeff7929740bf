#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_pcnn_gpu.py > gpurun_out/pcnn_t.log 2>&1; rc=$?
tail -40 gpurun_out/pcnn_t.log
exit $rc
