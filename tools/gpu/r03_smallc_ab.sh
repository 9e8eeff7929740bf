#!/bin/bash
# small-channel kernels before / after the batched staging (+ s1[0] fusion): per-launch trace of the
# image-channel convs alone (SVAE_TRACE_GEMM drains the stream around each gather), then the step A/B
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for l in sequential-variational-autoencoder_amd/libsvae_hip.so ab/old.so; do
  SVAE_LIB=$PWD/$l SVAE_TRACE_GEMM=1 timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-fp32 > gpurun_out/trace_b.log 2> gpurun_out/trace_e.log || { tail -20 gpurun_out/trace_e.log; exit 1; }
  echo "$l: $(grep -c GEMM gpurun_out/trace_e.log) traced launches"
  grep "cin 3 n 32" gpurun_out/trace_e.log | tail -8
done
bash tools/gpu/r02_libab.sh sequential-variational-autoencoder_amd/libsvae_hip.so ab/old.so
