#!/bin/bash
# c_pixelvae chain: GPU parity vs oracle/pixelvae.py, train / generate, full-size properties; the
# existing PixelCNN head tests
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r03_pvae}
timeout -k 10 900 python -u -m pytest tests/test_pixelvae_gpu.py tests/test_pcnn_gpu.py -x -v -s --timeout 400 --timeout-method thread > gpurun_out/${TAG}_tests.txt 2>&1; rc=$?
grep -E "passed|failed|FAILED|c_pixelvae small" gpurun_out/${TAG}_tests.txt | tail -8
[ $rc -ne 0 ] && { grep -E "^E " gpurun_out/${TAG}_tests.txt | head -30; exit 1; }
exit 0
