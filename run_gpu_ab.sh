#!/bin/bash
# A/B of weight-GEMM split policy (env knobs), bench only
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in "512 4" "256 4" "256 8" "128 8" "384 6"; do
  set -- $cfg
  SVAE_WH_TARGET=$1 SVAE_WH_MINCH=$2 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/ab_$1_$2.log 2>&1 || exit 1
done
