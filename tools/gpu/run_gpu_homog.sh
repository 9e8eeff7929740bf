#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_homog_gpu.py tests/test_infomax_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/homog.log 2>&1
rc=$?; echo rc=$rc >> gpurun_out/homog.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1
echo rc=$? >> gpurun_out/tests.log
