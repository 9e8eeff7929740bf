#!/bin/bash
# bench A/B over environment settings (interleaved, 2 rounds): r02_envab.sh "A=1" "B=2" ...
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in $(seq 1 ${ROUNDS:-2}); do
  for e in "X=0" "$@"; do
    env $e timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-fp32 > gpurun_out/envab_b.log 2>&1 || { tail -20 gpurun_out/envab_b.log; exit 1; }
    echo "$e bench $(tail -1 gpurun_out/envab_b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["elbo_per_img"], d["roofline"]["avg_launch_us"])')"
  done
done
