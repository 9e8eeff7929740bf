#!/bin/bash
# round 3, first call: headline parity printout of the round-start tree, fp32-mode kernel-trace
# stats (none since r01_v0), SQ counter passes of the bf16 bench command (halo_kw family)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r03_v0}
timeout -k 10 600 python -u -m pytest tests/test_headline_gpu.py -x -v -s --timeout 500 --timeout-method thread > gpurun_out/${TAG}_headline.txt 2>&1 || { tail -30 gpurun_out/${TAG}_headline.txt; exit 1; }
grep -A8 "headline CelebA" gpurun_out/${TAG}_headline.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_fp32prof -o run -- python3 bench.py --dtype fp32 --steps 5 --warmup 2 --no-cpu-baseline --no-fp32 > gpurun_out/${TAG}_fp32prof.log 2>&1 || { tail -20 gpurun_out/${TAG}_fp32prof.log; exit 1; }
tail -1 gpurun_out/${TAG}_fp32prof.log
python3 tools/prof_summary.py gpurun_out/${TAG}_fp32prof/run_results.db > gpurun_out/${TAG}_fp32_kernel_stats.txt 2>&1 || true
head -30 gpurun_out/${TAG}_fp32_kernel_stats.txt
rm -rf gpurun_out/${TAG}_fp32prof
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA --output-format csv -d gpurun_out/${TAG}_sq1 -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-fp32 > gpurun_out/${TAG}_sq1.log 2>&1 || exit 1
python3 tools/sq_summary.py gpurun_out/${TAG}_sq1 > gpurun_out/${TAG}_sq1.txt
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS --output-format csv -d gpurun_out/${TAG}_sq2 -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-fp32 > gpurun_out/${TAG}_sq2.log 2>&1 || exit 1
python3 tools/sq_summary.py gpurun_out/${TAG}_sq2 > gpurun_out/${TAG}_sq2.txt
rm -rf gpurun_out/${TAG}_sq1 gpurun_out/${TAG}_sq2
head -30 gpurun_out/${TAG}_sq1.txt; head -30 gpurun_out/${TAG}_sq2.txt
