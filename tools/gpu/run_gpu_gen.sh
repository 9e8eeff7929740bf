#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_generate_gpu.py tests/test_variants_gpu.py -q -x > gpurun_out/gen.log 2>&1
rc=$?; echo gen_rc=$rc >> gpurun_out/gen.log
exit $rc
