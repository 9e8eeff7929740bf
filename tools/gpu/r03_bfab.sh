#!/bin/bash
# c_pixelvae: bf16 output-gradient buffers on / off, two interleaved rounds, then a kernel profile (on)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
  for e in "X=0" "SVAE_PC_BF16_GRADS=0"; do
    env $e timeout -k 10 600 python bench.py --config c_pixelvae --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bfab.log 2>&1 || { tail -20 gpurun_out/bfab.log; exit 1; }
    echo "$e $(tail -1 gpurun_out/bfab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
bash tools/gpu/r03_pvprof.sh r03_pv6 > /dev/null 2>&1; head -14 gpurun_out/r03_pv6_kernel_stats.txt | cut -c1-150
