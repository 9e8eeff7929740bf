#!/bin/bash
# weight-gradient parity tests + profile + bench
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_wgrad_bf16_gpu.py tests/test_engine_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1
rc=$?; echo tests_rc=$rc >> gpurun_out/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bf16 -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/prof.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench.log 2>&1 || exit 1
