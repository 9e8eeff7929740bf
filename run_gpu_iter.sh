#!/bin/bash
# iteration run: op parity -> microbench -> in-situ -> full GPU suite + profile + bench
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gather_bf16_gpu.py -q -x > gpurun_out/ops.log 2>&1
rc=$?; echo ops_rc=$rc >> gpurun_out/ops.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python tools/bench_gather.py > gpurun_out/gb.log 2>&1 || exit 1
bash run_gpu.sh
