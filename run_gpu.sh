#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests/test_engine_gpu.py -q -x -s > gpurun_out/tests.log 2>&1
rc=$?; echo tests_rc=$rc >> gpurun_out/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bf16 -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --dtype bf16 > gpurun_out/prof.log 2>&1
echo prof_rc=$? >> gpurun_out/prof.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --dtype bf16 > gpurun_out/bench.log 2>&1
echo bench_rc=$? >> gpurun_out/bench.log
