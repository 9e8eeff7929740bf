#!/bin/bash
# GPU job: parity tests then a profiled bench.  Every GPU step has its own time limit;
# a fault/timeout ends the script.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests/test_engine_gpu.py -q -x > gpurun_out/engine.log 2>&1
rc=$?; echo eng_rc=$rc >> gpurun_out/engine.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof.log 2>&1
echo prof_rc=$? >> gpurun_out/prof.log
