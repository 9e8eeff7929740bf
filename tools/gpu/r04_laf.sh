#!/bin/bash
# last-arriver BN finalisation (SVAE_BN_LAF): its bitwise test, parity suites, then the bench A/B
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_fused_adam_gpu.py -x -q -k last_arriver --timeout 300 --timeout-method thread > gpurun_out/r04_laf_bitwise.txt 2>&1 || { tail -40 gpurun_out/r04_laf_bitwise.txt; exit 1; }
tail -1 gpurun_out/r04_laf_bitwise.txt
timeout -k 10 900 python -u -m pytest tests/test_engine_gpu.py tests/test_golden_gpu.py tests/test_halo_gpu.py tests/test_fused_adam_gpu.py -x -q --timeout 600 --timeout-method thread > gpurun_out/r04_laf_tests.txt 2>&1 || { tail -40 gpurun_out/r04_laf_tests.txt; exit 1; }
tail -1 gpurun_out/r04_laf_tests.txt
ROUNDS=2 bash tools/gpu/r04_ab.sh SVAE_BN_LAF=0 SVAE_BN_LAF=1 SVAE_FOLD=1
