#!/bin/bash
# split-latent step 0 on the main stream vs on st3: GPU suite, A/B bench, then a profile
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
for rep in 1 2; do
for v in "" "SVAE_SFC0_SIDE=1"; do
  env $v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/ab.json 2>gpurun_out/ab.err || exit 1
  echo "[$v] $(python -c "import json;d=json.load(open('gpurun_out/ab.json'));print(d['ms_per_step'],d['value'])")"
done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bf16 -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/prof.log 2>&1 || exit 1
