#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do for v in "4 2048" "2 2048" "1 2048" "2 4096" "1 8192"; do
  set -- $v
  SVAE_AP_RPT=$1 SVAE_AP_CAP=$2 timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-fp32 > gpurun_out/rpt_b.log 2>&1 || exit 1
  echo "RPT=$1 CAP=$2 $(tail -1 gpurun_out/rpt_b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["elbo_per_img"])')"
done; done
