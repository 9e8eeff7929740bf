#!/bin/bash
# BN finalise-once (SVAE_BN_FIN): bitwise test, then interleaved A/B in both modes
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_fused_adam_gpu.py -k finalise_once -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05_fin_tests.txt 2>&1 || { tail -30 gpurun_out/r05_fin_tests.txt; exit 1; }
tail -2 gpurun_out/r05_fin_tests.txt
ROUNDS=2 STEPS=30 bash tools/gpu/ab.sh SVAE_BN_FIN=1 || exit 1
ROUNDS=2 STEPS=30 BENCH_ARGS="--dtype bf16" bash tools/gpu/ab.sh SVAE_BN_FIN=1
