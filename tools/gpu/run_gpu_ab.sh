#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
for n in 0 64 128 192; do
  SVAE_SIDE_CUS=$n timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/cu_${n}_$rep.log 2>&1 || exit 1
done; done
