#!/bin/bash
# bf16 pre-BN storage: the fold's bitwise test with it, kernel stats with / without it (SVAE_PRE_F32=1),
# then the bench A/B of bf16 pre, fp32 pre, and the fold on top of bf16 pre
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_fused_adam_gpu.py -x -q -k "fold" --timeout 300 --timeout-method thread > gpurun_out/r04_pre2_tests.txt 2>&1 || { tail -30 gpurun_out/r04_pre2_tests.txt; exit 1; }
tail -1 gpurun_out/r04_pre2_tests.txt
Q="--no-cpu-baseline --no-fp32 --steps 10 --warmup 3"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pp_a -o run -- python3 bench.py $Q > gpurun_out/pp_a.log 2>&1 || exit 1
python3 tools/prof_summary.py gpurun_out/pp_a/run_results.db > gpurun_out/r04_pre_bf16pre_kernel_stats.txt 2>&1; rm -rf gpurun_out/pp_a
SVAE_PRE_F32=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pp_b -o run -- python3 bench.py $Q > gpurun_out/pp_b.log 2>&1 || exit 1
python3 tools/prof_summary.py gpurun_out/pp_b/run_results.db > gpurun_out/r04_pre_f32pre_kernel_stats.txt 2>&1; rm -rf gpurun_out/pp_b
ROUNDS=2 bash tools/gpu/r04_ab.sh SVAE_PRE_F32=1 SVAE_FOLD=1
