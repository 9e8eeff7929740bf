#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_headline_gpu.py tests/test_engine_gpu.py tests/test_chain_variants_gpu.py tests/test_generate_gpu.py tests/test_golden_gpu.py tests/test_infomax_gpu.py tests/test_gather_bf16_gpu.py tests/test_halo_gpu.py > gpurun_out/misc_t.log 2>&1 || { tail -20 gpurun_out/misc_t.log; exit 1; }
tail -1 gpurun_out/misc_t.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-fp32 > gpurun_out/misc_b$i.log 2>&1 || exit 1
  echo "bench $(tail -1 gpurun_out/misc_b$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["elbo_per_img"])')"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/misc_prof -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-fp32 > gpurun_out/misc_prof.log 2>&1 || exit 1
python3 tools/prof_summary.py gpurun_out/misc_prof/run_results.db > gpurun_out/misc_kernel_stats.txt 2>&1 || true
grep -E "colsum|latent_fwd|splitfc_bwd|splitfc_dz" gpurun_out/misc_kernel_stats.txt | cut -c1-60,110-175
