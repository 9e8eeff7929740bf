#!/bin/bash
# narrow recognition heads, forward recognition split, batched small-channel staging: parity subset,
# then the bench A/B and a kernel-trace of the default step
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_fused_adam_gpu.py tests/test_engine_gpu.py tests/test_golden_gpu.py tests/test_ops_gpu.py -x -q -s --timeout 300 --timeout-method thread > gpurun_out/heads_tests.txt 2>&1 || { tail -30 gpurun_out/heads_tests.txt; exit 1; }
tail -2 gpurun_out/heads_tests.txt; grep "rec split" gpurun_out/heads_tests.txt
SVAE_REC_SPLIT=1 timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_headline_gpu.py -x -q --timeout 500 --timeout-method thread > gpurun_out/recsplit_tests.txt 2>&1 || { tail -30 gpurun_out/recsplit_tests.txt; exit 1; }
tail -1 gpurun_out/recsplit_tests.txt
bash tools/gpu/r02_envab.sh SVAE_HEADS_SKINNY=1 SVAE_REC_SPLIT=1 SVAE_NO_BWFUSE_OUT=1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/h_prof -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-fp32 > gpurun_out/h_prof.log 2>&1 || exit 1
python3 tools/prof_summary.py gpurun_out/h_prof/run_results.db > gpurun_out/h_kernel_stats.txt 2>&1 || true
python3 tools/stream_breakdown.py gpurun_out/h_prof/run_results.db 28 20 8 > gpurun_out/h_streams.txt 2>&1 || true
rm -rf gpurun_out/h_prof
head -4 gpurun_out/h_streams.txt
