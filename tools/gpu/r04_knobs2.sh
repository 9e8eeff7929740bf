#!/bin/bash
# split-target sweep around the new split-mode default (128): larger targets for bf16x6, 128 for bf16
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
ROUNDS=2 bash tools/gpu/r04_ab.sh SVAE_WH2_TARGET=192 SVAE_WH2_TARGET=256 SVAE_WH2_TARGET=96
