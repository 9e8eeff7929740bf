#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu/run_gpu.sh || exit 1
SVAE_NO_SIDE=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_noside.log 2>&1
