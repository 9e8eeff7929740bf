#!/bin/bash
# probe-overhead A/B: every dominant-kernel launch timed vs the first 96
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do for p in 0 96; do
  timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-fp32 --probe-launches $p > gpurun_out/pr_b.log 2>&1 || exit 1
  echo "probe=$p $(tail -1 gpurun_out/pr_b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], r["avg_launch_us"], r["frac"], r["launches_per_step"])')"
done; done
