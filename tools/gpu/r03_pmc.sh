#!/bin/bash
# bf16 bench command: per-GEMM trace (one step, stream drained around each gather-GEMM), PMC
# FETCH / WRITE passes (calibrated rules of tools/pmc_traffic.py), kernel-trace stats + streams
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r03_v2}
SVAE_TRACE_GEMM=1 timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-fp32 > gpurun_out/${TAG}_trace_gemm.log 2>&1 || { tail -5 gpurun_out/${TAG}_trace_gemm.log; exit 1; }
grep -c GEMM gpurun_out/${TAG}_trace_gemm.log
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_pmc_fetch -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-fp32 > gpurun_out/${TAG}_pmc_fetch.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${TAG}_pmc_write -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-fp32 > gpurun_out/${TAG}_pmc_write.log 2>&1 || exit 1
python3 tools/pmc_traffic.py gpurun_out/${TAG}_pmc_fetch gpurun_out/${TAG}_pmc_write gpurun_out/${TAG}_pmc_traffic.json $TAG > gpurun_out/${TAG}_pmc.txt; rm -rf gpurun_out/${TAG}_pmc_fetch gpurun_out/${TAG}_pmc_write
head -30 gpurun_out/${TAG}_pmc.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-fp32 > gpurun_out/${TAG}_prof.log 2>&1 || exit 1
python3 tools/prof_summary.py gpurun_out/${TAG}_prof/run_results.db > gpurun_out/${TAG}_kernel_stats.txt 2>&1 || true
python3 tools/stream_breakdown.py gpurun_out/${TAG}_prof/run_results.db > gpurun_out/${TAG}_streams.txt 2>&1 || true
rm -rf gpurun_out/${TAG}_prof
head -8 gpurun_out/${TAG}_streams.txt
