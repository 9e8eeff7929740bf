#!/bin/bash
# side stream on a CU subset: parity subset with the mask on, then bench A/B on a non-default stream
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
SVAE_SIDE_CUMASK=4 timeout -k 10 600 python -u -m pytest tests/test_fused_adam_gpu.py tests/test_golden_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/cumask_tests.txt 2>&1 || { tail -30 gpurun_out/cumask_tests.txt; exit 1; }
tail -1 gpurun_out/cumask_tests.txt
bash tools/gpu/r02_envab.sh "SVAE_BENCH_STREAM=1" "SVAE_BENCH_STREAM=1 SVAE_SIDE_CUMASK=4" "SVAE_BENCH_STREAM=1 SVAE_SIDE_CUMASK=8" "SVAE_BENCH_STREAM=1 SVAE_SIDE_CUMASK=2"
