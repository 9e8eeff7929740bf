#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_wgrad_bf16_gpu.py -q -x > gpurun_out/wg.log 2>&1
rc=$?; echo wg_rc=$rc >> gpurun_out/wg.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/gpu/run_gpu.sh
