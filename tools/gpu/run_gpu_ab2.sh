#!/bin/bash
# GPU suite, then A/B of the stream placement knobs (same process order, one device)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
for rep in 1 2; do
for v in "" "SVAE_ADAM_ST2=1" "SVAE_SFC_ALL=1" "SVAE_ADAM_ST2=1 SVAE_SFC_ALL=1"; do
  env $v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/ab.json 2>gpurun_out/ab.err || exit 1
  echo "[$v] $(python -c "import json;d=json.load(open('gpurun_out/ab.json'));print(d['ms_per_step'],d['value'])")"
done
done
