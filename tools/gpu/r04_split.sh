cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
SVAE_KW_SPLIT_BM=32 timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -q -k bf16x6 --timeout 300 --timeout-method thread > gpurun_out/r04_split_tests.txt 2>&1 || { tail -30 gpurun_out/r04_split_tests.txt; exit 1; }
tail -1 gpurun_out/r04_split_tests.txt
bash tools/gpu/r04_ab.sh SVAE_KW_SPLIT_BM=32 SVAE_KW_PI3=0 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04_p6 -o run -- python3 bench.py --dtype bf16x6 --steps 6 --warmup 2 --no-cpu-baseline --no-fp32 > gpurun_out/r04_p6.log 2>&1 || exit 1
python3 tools/prof_summary.py gpurun_out/r04_p6/run_results.db > gpurun_out/r04_x6_kernel_stats.txt 2>&1 || true
python3 tools/stream_breakdown.py gpurun_out/r04_p6/run_results.db 28 6 4 > gpurun_out/r04_x6_streams.txt 2>&1 || true
rm -rf gpurun_out/r04_p6
head -32 gpurun_out/r04_x6_streams.txt
