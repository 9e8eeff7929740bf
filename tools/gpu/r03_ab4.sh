#!/bin/bash
# FC BN-backward fusion variant: parity subset, then the step A/B
# (knob on vs off)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
SVAE_BWFUSE_FC=1 timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_golden_gpu.py tests/test_headline_gpu.py -x -q --timeout 500 --timeout-method thread > gpurun_out/fc_tests.txt 2>&1 || { tail -30 gpurun_out/fc_tests.txt; exit 1; }
tail -1 gpurun_out/fc_tests.txt
bash tools/gpu/r02_envab.sh SVAE_BWFUSE_FC=1
