#!/bin/bash
# per-layer isolated gather-GEMM times (SVAE_TRACE_GEMM=1) of one bench step, bf16 and bf16x6
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r04_trace}
for dt in bf16 bf16x6; do
  SVAE_TRACE_GEMM=1 timeout -k 10 300 python bench.py --dtype $dt --steps 1 --warmup 1 --no-cpu-baseline --no-fp32 > gpurun_out/${TAG}_${dt}.out 2> gpurun_out/${TAG}_${dt}.err || { tail -20 gpurun_out/${TAG}_${dt}.err; exit 1; }
  python tools/trace_summary.py gpurun_out/${TAG}_${dt}.err > gpurun_out/${TAG}_${dt}.txt
  head -40 gpurun_out/${TAG}_${dt}.txt
done
