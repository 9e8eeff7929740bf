#!/bin/bash
# BN accumulator shard cap and apply-pass block budget (the per-block statistics gather volume)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
ROUNDS=2 bash tools/gpu/r04_ab.sh ${@:-SVAE_BN_SHMAX=4 SVAE_BN_SHMAX=8 SVAE_AP_CAP=2048 SVAE_BN_SHMAX=4,SVAE_AP_CAP=2048}
