#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_engine_gpu.py -q -x -k "bf16" -s > gpurun_out/tests.log 2>&1
rc=$?; echo tests_rc=$rc >> gpurun_out/tests.log
