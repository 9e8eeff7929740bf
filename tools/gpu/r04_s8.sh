#!/bin/bash
# split-plane staging in value pairs (opload.h split8): bitwise (same elbo), timing against the previous
# build (abl/s8old.so through SVAE_LIB)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_golden_gpu.py -x -q -k "bf16x6 or split" --timeout 300 --timeout-method thread > gpurun_out/r04_s8_tests.txt 2>&1 || { tail -30 gpurun_out/r04_s8_tests.txt; exit 1; }
tail -1 gpurun_out/r04_s8_tests.txt
ROUNDS=3 bash tools/gpu/r04_ab.sh X=1@abl/s8old.so
