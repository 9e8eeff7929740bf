#!/bin/bash
# iteration run: op parity (new kernels first) -> full GPU suite + profile + bench
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_ops_gpu.py tests/test_gather_bf16_gpu.py -q -x > gpurun_out/ops.log 2>&1
rc=$?; echo ops_rc=$rc >> gpurun_out/ops.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/gpu/run_gpu.sh "$@"
