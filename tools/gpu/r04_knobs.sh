#!/bin/bash
# knob sweep for the parity mode (bf16x6) on the final tree: weight-GEMM split targets, dense split-K target
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
ROUNDS=2 bash tools/gpu/r04_ab.sh SVAE_WH2_TARGET=128 SVAE_WH2_MINCH=2 SVAE_WH_TARGET=512 SVAE_DKW_TGT=1024
