#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gather_bf16_gpu.py -q -x > gpurun_out/ops.log 2>&1
rc=$?; echo ops_rc=$rc >> gpurun_out/ops.log
exit $rc
