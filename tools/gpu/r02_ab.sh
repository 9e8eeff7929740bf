#!/bin/bash
# in-situ A/B of the stride-1 weight-GEMM variants (env knobs), two interleaved rounds
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for round in 1 2; do
for v in "SVAE_NO_WH2=1" "SVAE_WH2_DB=1" "SVAE_WH2_DB=0" "SVAE_WH2_KYR=2" "SVAE_WH2_KYR=2 SVAE_WH2_DB=0" "SVAE_WH2_TARGET=128"; do
  env $v timeout -k 10 120 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-fp32 > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); r=d['roofline']
print('%-32s %8.3f ms/step %8.1f img/s  probe %6.2f us frac %.4f' % (sys.argv[1], d['ms_per_step'], d['value'], r['avg_launch_us'], r['frac']))" "$v"
done
done
