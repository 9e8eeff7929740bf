#!/bin/bash
# bitwise A/B of an engine switch (tools/dpre_bitwise.py), then a bench per setting
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
VAR=$1
timeout -k 10 300 python3 tools/dpre_bitwise.py celeba 32 $VAR > gpurun_out/bitab.txt 2>&1; echo "bitwise rc=$?"; tail -2 gpurun_out/bitab.txt
for i in 1 2; do
  for e in "X=0" "$VAR"; do
    env $e timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-fp32 > gpurun_out/bitab_b.log 2>&1 || { tail -20 gpurun_out/bitab_b.log; exit 1; }
    echo "$e bench $(tail -1 gpurun_out/bitab_b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["elbo_per_img"])')"
  done
done
