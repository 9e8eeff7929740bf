#!/bin/bash
# A/B of an env switch on the bench (alternating, same box): run_gpu_ab.sh VAR VALUE_A VALUE_B
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
V=$1; A=$2; B=$3
for i in 1 2 3; do
  env $V=$A timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/ab_a$i.log 2>&1 || exit 1
  env $V=$B timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/ab_b$i.log 2>&1 || exit 1
done
