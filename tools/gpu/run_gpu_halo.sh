#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_halo_gpu.py -q -x -s > gpurun_out/halo.log 2>&1
rc=$?; echo halo_rc=$rc >> gpurun_out/halo.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/gpu/run_gpu.sh
