#!/bin/bash
# per-layer gather-GEMM timings (SVAE_TRACE_GEMM) of one bench step
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
SVAE_TRACE_GEMM=1 timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-fp32 > gpurun_out/trace.log 2> gpurun_out/trace.err || { tail -20 gpurun_out/trace.err; exit 1; }
grep -c GEMM gpurun_out/trace.err
