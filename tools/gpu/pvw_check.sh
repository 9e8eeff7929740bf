#!/bin/bash
# the head's fused-plane weight gradients: parity suites, then c_pixelvae A/B against the three-launch form
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/gpu/pv_ab.sh SVAE_PC_HP 0
