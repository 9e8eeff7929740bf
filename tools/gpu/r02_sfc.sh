#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do for v in 1 0; do
  SVAE_SFC=$v timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-fp32 > gpurun_out/sfc_b$v.log 2>&1 || exit 1
  echo "SFC=$v $(tail -1 gpurun_out/sfc_b$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done; done
