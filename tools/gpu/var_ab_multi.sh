#!/bin/bash
# interleaved A/B of the shipping library against several compile-time variants (expt/<name>.so each)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
specs=()
for v in "$@"; do specs+=("V_$v=1@expt/$v.so"); done
ROUNDS=${ROUNDS:-2} STEPS=30 bash tools/gpu/ab.sh "D=1@sequential-variational-autoencoder_amd/libsvae_hip.so" "${specs[@]}"
