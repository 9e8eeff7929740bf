#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 0 1 0 1; do
  echo "SVAE_HALO_1BUF=$v"; SVAE_HALO_1BUF=$v timeout -k 10 120 python tools/bench_gather.py 1 || exit 1
done
for v in 0 1 0 1; do
  SVAE_HALO_1BUF=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fp32 > gpurun_out/h1b_$v.log 2>&1 || exit 1
  echo "1BUF=$v $(tail -1 gpurun_out/h1b_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
