#!/bin/bash
# GPU job: parity tests then bench.  Each GPU step has its own time limit; stop on fault/timeout.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests/test_ops_gpu.py tests/test_engine_gpu.py -q -x > gpurun_out/tests.log 2>&1
rc=$?; echo tests_rc=$rc >> gpurun_out/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench.log 2>&1
echo bench_rc=$? >> gpurun_out/bench.log
