#!/bin/bash
# chain variants (f3) on the GPU: new tests first, then the existing suite's variant tests
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread tests/test_chain_variants_gpu.py > gpurun_out/r02_f3.log 2>&1
rc=$?; echo rc=$rc; grep -E "passed|failed|rel|Error|error" gpurun_out/r02_f3.log | tail -40
exit $rc
