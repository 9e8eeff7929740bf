#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_headline_gpu.py tests/test_engine_gpu.py tests/test_chain_variants_gpu.py tests/test_generate_gpu.py tests/test_golden_gpu.py tests/test_infomax_gpu.py tests/test_homog_gpu.py tests/test_train_api_gpu.py tests/test_pcnn_gpu.py tests/test_gather_bf16_gpu.py > gpurun_out/dkw_t.log 2>&1 || { tail -30 gpurun_out/dkw_t.log; exit 1; }
tail -1 gpurun_out/dkw_t.log
for r in 1 2; do for v in 0 1; do
  SVAE_NO_DKW=$v timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-fp32 > gpurun_out/dkw_b$v.log 2>&1 || exit 1
  echo "NO_DKW=$v $(tail -1 gpurun_out/dkw_b$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["elbo_per_img"])')"
done; done
