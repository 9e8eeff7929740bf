#!/bin/bash
# row-group recognition-heads backward: its check against the one-k-per-thread kernel, then the bench A/B
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_heads_gpu.py -x -q -s --timeout 250 --timeout-method thread > gpurun_out/r04_heads_test.txt 2>&1 || { tail -30 gpurun_out/r04_heads_test.txt; exit 1; }
grep "re-associated\|passed" gpurun_out/r04_heads_test.txt
ROUNDS=2 bash tools/gpu/r04_ab.sh SVAE_HEADS_RG=0
