#!/bin/bash
# persistent halo_kw: bf16 parity test with it on, then an interleaved bench A/B
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
SVAE_KW_PERSIST=1 timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -k "bf16_mode or full_size or celeba_geometry" -x -q --timeout 300 --timeout-method thread > gpurun_out/persist_tests.txt 2>&1 || { grep -E "^E |FAILED" gpurun_out/persist_tests.txt | head; tail -3 gpurun_out/persist_tests.txt; exit 1; }
tail -1 gpurun_out/persist_tests.txt
ROUNDS=2 bash tools/gpu/r02_envab.sh "SVAE_KW_PERSIST=1" "SVAE_KW_PERSIST=2"
