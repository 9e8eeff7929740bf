#!/bin/bash
# A/B: output-operand packing ahead of the recognition pass (default) vs the former place, the
# weight-GEMM split target, hardware queues; then the kernel trace of the default for the step-start gap
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r03_ab2}
ROUNDS=2 bash tools/gpu/r02_envab.sh "SVAE_PACK_LATE=1" "SVAE_WH2_TARGET=64" "GPU_MAX_HW_QUEUES=8" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-fp32 > gpurun_out/${TAG}_prof.log 2>&1 || exit 1
python3 tools/stream_breakdown.py gpurun_out/${TAG}_prof/run_results.db 28 20 8 > gpurun_out/${TAG}_streams.txt 2>&1 || true
grep -A 8 "main stream" gpurun_out/${TAG}_streams.txt
