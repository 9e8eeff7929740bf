#!/bin/bash
# side-stream batching parity + env A/B, then the write-through-store library A/B (with its parity subset)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
SB=3 bash tools/gpu/r03_sideab.sh SVAE_SIDE_BATCH=3 SVAE_SIDE_BATCH=100 SVAE_PACK_FIRST=1 || exit 1
SVAE_LIB=$PWD/ab/wt.so timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py tests/test_golden_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/wt_tests.txt 2>&1 || { tail -30 gpurun_out/wt_tests.txt; exit 1; }
tail -2 gpurun_out/wt_tests.txt
bash tools/gpu/r02_libab.sh sequential-variational-autoencoder_amd/libsvae_hip.so ab/wt.so
