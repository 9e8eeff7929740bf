#!/bin/bash
# interleaved A/B of the shipping library against one compile-time variant (expt/$1.so), both modes
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
ROUNDS=${ROUNDS:-2} STEPS=30 bash tools/gpu/ab.sh "D=1@sequential-variational-autoencoder_amd/libsvae_hip.so" "V=1@expt/$1.so" || exit 1
[ -n "$BF16" ] && ROUNDS=${ROUNDS:-2} STEPS=30 BENCH_ARGS="--dtype bf16" bash tools/gpu/ab.sh "D=1@sequential-variational-autoencoder_amd/libsvae_hip.so" "V=1@expt/$1.so"
exit 0
