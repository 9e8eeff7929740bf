#!/bin/bash
# halo2 weight-GEMM: parity on the CelebA layer shapes, then microbench A/B (path 2 new / 3 old) + knobs
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_wgrad_bf16_gpu.py > gpurun_out/r02_wh2_tests.log 2>&1 || { tail -40 gpurun_out/r02_wh2_tests.log; exit 1; }
tail -2 gpurun_out/r02_wh2_tests.log
echo "== path 3 (old halo)"; timeout -k 10 120 python tools/bench_wgrad.py 30 3 || exit 1
echo "== path 2 (halo2 default)"; timeout -k 10 120 python tools/bench_wgrad.py 30 2 || exit 1
echo "== KYR=2"; SVAE_WH2_KYR=2 timeout -k 10 120 python tools/bench_wgrad.py 30 2 | head -6 || exit 1
echo "== TARGET=128"; SVAE_WH2_TARGET=128 timeout -k 10 120 python tools/bench_wgrad.py 30 2 | head -6 || exit 1
echo "== TARGET=512"; SVAE_WH2_TARGET=512 timeout -k 10 120 python tools/bench_wgrad.py 30 2 | head -6 || exit 1
echo "== MINCH=8"; SVAE_WH2_MINCH=8 timeout -k 10 120 python tools/bench_wgrad.py 30 2 | head -6 || exit 1
