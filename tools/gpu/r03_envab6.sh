#!/bin/bash
# bench A/B over environment settings for one dtype (interleaved, ROUNDS rounds): DT=bf16x6 r03_envab6.sh "A=1" ...
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in $(seq 1 ${ROUNDS:-2}); do
  for e in "X=0" "$@"; do
    env $e timeout -k 10 240 python bench.py --dtype ${DT:-bf16x6} --steps ${STEPS:-20} --warmup 4 --no-cpu-baseline --no-fp32 > gpurun_out/envab6_b.log 2>&1 || { tail -20 gpurun_out/envab6_b.log; exit 1; }
    echo "$e bench $(tail -1 gpurun_out/envab6_b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["elbo_per_img"])')"
  done
done
