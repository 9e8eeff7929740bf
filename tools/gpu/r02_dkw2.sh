#!/bin/bash
# dense FC GEMM split knobs A/B (two interleaved rounds)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do for v in "512 8" "1024 8" "512 4" "1024 4" "256 8" "512 16"; do
  set -- $v
  SVAE_DKW_TGT=$1 SVAE_DKW_MINK=$2 timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-fp32 > gpurun_out/dkw2.log 2>&1 || exit 1
  echo "TGT=$1 MINK=$2 $(tail -1 gpurun_out/dkw2.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done; done
