#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/tests.log 2>&1
rc=$?; echo tests_rc=$rc >> gpurun_out/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --config lsun --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_lsun.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config lsun --dtype fp32 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_lsun32.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --dtype fp32 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_cel32.log 2>&1 || exit 1
