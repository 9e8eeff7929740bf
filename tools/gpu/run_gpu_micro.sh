#!/bin/bash
# gather microbench A/B on SVAE_HALO_FILL + benches
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
SVAE_HALO_FILL=256 timeout -k 10 300 python tools/bench_gather.py 2 > gpurun_out/micro.log 2>&1 || exit 1
timeout -k 10 300 python tools/bench_gather.py 2 > gpurun_out/micro_b.log 2>&1 || exit 1
SVAE_HALO_FILL=256 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_b.log 2>&1 || exit 1
SVAE_HALO_FILL=1024 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_c.log 2>&1 || exit 1
