#!/bin/bash
# split-mode small-C weight gradients (engine parity at the CelebA geometry), c_pixelvae tests, the
# c_pixelvae bench leg, and the default bench line (parity_value)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r03_v2}
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_pixelvae_gpu.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.txt 2>&1; rc=$?
grep -E "passed|failed|FAILED|c_pixelvae small" gpurun_out/${TAG}_tests.txt | tail -6
[ $rc -ne 0 ] && { grep -E "^E " gpurun_out/${TAG}_tests.txt | head -30; exit 1; }
timeout -k 10 600 python bench.py --config c_pixelvae --steps 5 --warmup 2 > gpurun_out/${TAG}_pvae_bench.log 2>&1 || { tail -20 gpurun_out/${TAG}_pvae_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_pvae_bench.log
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log | cut -c1-700
