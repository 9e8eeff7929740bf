#!/bin/bash
# c_pixelvae weight-gradient split targets A/B (two interleaved rounds)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
  for e in "X=0" "SVAE_PW_TARGET=1024" "SVAE_PW4_TARGET=512" "SVAE_PW_TARGET=1024 SVAE_PW4_TARGET=512" "SVAE_PW_TARGET=4096 SVAE_PW4_TARGET=2048"; do
    env $e timeout -k 10 600 python bench.py --config c_pixelvae --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/pwt.log 2>&1 || { tail -20 gpurun_out/pwt.log; exit 1; }
    echo "$e $(tail -1 gpurun_out/pwt.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
