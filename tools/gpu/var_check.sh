#!/bin/bash
# a compile-time variant (expt/$1.so): the split-mode gather / engine parity tests on it, then the
# interleaved bench A/B against the shipping library
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_split_gather_gpu.py \
  > gpurun_out/var_default_tests.txt 2>&1 || { tail -30 gpurun_out/var_default_tests.txt; exit 1; }
tail -1 gpurun_out/var_default_tests.txt
SVAE_LIB=$PWD/expt/$1.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_split_gather_gpu.py tests/test_headline_gpu.py tests/test_engine_gpu.py > gpurun_out/var_$1_tests.txt 2>&1 || { tail -30 gpurun_out/var_$1_tests.txt; exit 1; }
tail -2 gpurun_out/var_$1_tests.txt
bash tools/gpu/var_ab.sh $1 2>&1 | tee gpurun_out/var_$1_ab.txt
