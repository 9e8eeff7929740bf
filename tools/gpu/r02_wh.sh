#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for t in 128 256 512; do echo "WH2_TARGET=$t"; SVAE_WH2_TARGET=$t timeout -k 10 120 python tools/bench_wgrad.py 20 | head -6; done
for t in 128 256 512 128 256; do
  SVAE_WH2_TARGET=$t timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fp32 > gpurun_out/wh_b$t.log 2>&1 || exit 1
  echo "WH2_TARGET=$t $(tail -1 gpurun_out/wh_b$t.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], r["avg_launch_us"], r["frac"])')"
done
