#!/bin/bash
# small-channel conv with an fp32-only y read path in its fused BN epilogue: parity spot check, then the
# CelebA bench A/B against the previous build (abl/pre_sc.so; same elbo = bitwise) and its kernel time
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_golden_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_sc_tests.txt 2>&1 || { tail -30 gpurun_out/r04_sc_tests.txt; exit 1; }
tail -1 gpurun_out/r04_sc_tests.txt
ROUNDS=3 bash tools/gpu/r04_ab.sh X=1@abl/pre_sc.so
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/sc_p -o run -- python3 bench.py --no-cpu-baseline --no-fp32 --steps 10 --warmup 3 > gpurun_out/sc_p.log 2>&1 || exit 1
python3 tools/prof_summary.py gpurun_out/sc_p/run_results.db > gpurun_out/r04_sc_kernel_stats.txt 2>&1; rm -rf gpurun_out/sc_p
grep conv_smallc gpurun_out/r04_sc_kernel_stats.txt
