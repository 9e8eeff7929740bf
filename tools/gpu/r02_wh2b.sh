#!/bin/bash
# halo2 weight-GEMM: kernel-only times (rocprof) for KYR 4 / 2, and SQ counters
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r02_wh2_k4 -o run -- python3 tools/bench_wgrad.py 20 2 > gpurun_out/r02_wh2_k4.log 2>&1 || exit 1
SVAE_WH2_KYR=2 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r02_wh2_k2 -o run -- python3 tools/bench_wgrad.py 20 2 > gpurun_out/r02_wh2_k2.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA --output-format csv -d gpurun_out/r02_wh2_sq1 -o run -- python3 tools/bench_wgrad.py 3 2 > gpurun_out/r02_wh2_sq1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r02_wh2_fetch -o run -- python3 tools/bench_wgrad.py 3 2 > gpurun_out/r02_wh2_fetch.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r02_wh2_write -o run -- python3 tools/bench_wgrad.py 3 2 > gpurun_out/r02_wh2_write.log 2>&1 || exit 1
python tools/sq_summary.py gpurun_out/r02_wh2_sq1 | head -12
python tools/pmc_traffic.py gpurun_out/r02_wh2_fetch gpurun_out/r02_wh2_write gpurun_out/r02_wh2_traffic.json wh2 | head -12
