#!/bin/bash
# bf16 concat buffers: bitwise against fp32 storage, then the bench A/B
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_fused_adam_gpu.py -x -q -k concat --timeout 300 --timeout-method thread > gpurun_out/r04_cat_tests.txt 2>&1 || { tail -30 gpurun_out/r04_cat_tests.txt; exit 1; }
tail -1 gpurun_out/r04_cat_tests.txt
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_golden_gpu.py tests/test_halo_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_cat_tests2.txt 2>&1 || { tail -30 gpurun_out/r04_cat_tests2.txt; exit 1; }
tail -1 gpurun_out/r04_cat_tests2.txt
ROUNDS=2 bash tools/gpu/r04_ab.sh SVAE_CAT_F32=1
