#!/bin/bash
# session-2 batch: FC BN-backward fusion variant (parity subset + step A/B), small-channel staging
# before / after (trace + step A/B), parity-mode knobs
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
SVAE_LIB=$PWD/ab/fc.so timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_golden_gpu.py tests/test_headline_gpu.py -x -q --timeout 500 --timeout-method thread > gpurun_out/fc_tests.txt 2>&1 || { tail -30 gpurun_out/fc_tests.txt; exit 1; }
tail -1 gpurun_out/fc_tests.txt
bash tools/gpu/r02_libab.sh sequential-variational-autoencoder_amd/libsvae_hip.so ab/fc.so ab/old.so || exit 1
for l in sequential-variational-autoencoder_amd/libsvae_hip.so ab/old.so; do
  SVAE_LIB=$PWD/$l SVAE_TRACE_GEMM=1 timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-fp32 > gpurun_out/trace_b.log 2> gpurun_out/trace_e.log || { tail -20 gpurun_out/trace_e.log; exit 1; }
  echo "$l:"; grep "cin 3 n 32" gpurun_out/trace_e.log | tail -4
done
DT=bf16x6 ROUNDS=1 bash tools/gpu/r03_envab6.sh SVAE_WH2_TARGET=32 SVAE_WH2_TARGET=128 SVAE_KW_BM=32
