#!/bin/bash
# bench A/B over library builds (interleaved, 2 rounds): r02_libab.sh ab/a.so ab/b.so ...
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
  for l in "$@"; do
    SVAE_LIB=$PWD/$l timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-fp32 > gpurun_out/libab_b.log 2>&1 || { tail -20 gpurun_out/libab_b.log; exit 1; }
    echo "$l bench $(tail -1 gpurun_out/libab_b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["elbo_per_img"], d["roofline"]["avg_launch_us"])')"
  done
done
