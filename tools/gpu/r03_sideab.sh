#!/bin/bash
# side-stream batching: parity subset with the knob on, then the interleaved bench A/B
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
SVAE_SIDE_BATCH=${SB:-3} timeout -k 10 600 python -u -m pytest tests/test_fused_adam_gpu.py tests/test_engine_gpu.py tests/test_dp_overlap_gpu.py tests/test_golden_gpu.py tests/test_chain_variants_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/sideab_tests.txt 2>&1 || { tail -30 gpurun_out/sideab_tests.txt; exit 1; }
tail -2 gpurun_out/sideab_tests.txt
bash tools/gpu/r02_envab.sh "$@"
