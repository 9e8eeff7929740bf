#!/bin/bash
# A/B: bench with and without a feature switch (env var given as $1)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/ab_on.log 2>&1 || exit 1
env $1=1 timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/ab_off.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/ab_on2.log 2>&1 || exit 1
env $1=1 timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/ab_off2.log 2>&1 || exit 1
