#!/bin/bash
# bf16-stored pre-BN conv outputs: parity suites touched by it, then the bench A/B against SVAE_PRE_F32=1
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_halo_gpu.py tests/test_engine_gpu.py tests/test_golden_gpu.py tests/test_headline_gpu.py -x -q -s --timeout 600 --timeout-method thread -k "not dp8" > gpurun_out/r04_pre_tests.txt 2>&1 || { tail -40 gpurun_out/r04_pre_tests.txt; exit 1; }
tail -1 gpurun_out/r04_pre_tests.txt
grep -i "gradients vs float64\|worst" gpurun_out/r04_pre_tests.txt | head -5
ROUNDS=2 bash tools/gpu/r04_ab.sh SVAE_PRE_F32=1
