#!/bin/bash
# dense FC GEMM: K-interleave width (SVAE_DKW_WK) A/B + per-shape kernel times
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for wk in 1 2 4; do
SVAE_DKW_WK=$wk timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_headline_gpu.py tests/test_pcnn_gpu.py -k "not full_size" > gpurun_out/d3_t.log 2>&1 || { tail -30 gpurun_out/d3_t.log; exit 1; }
echo "WK=$wk $(tail -1 gpurun_out/d3_t.log)"
done
for r in 1 2; do for wk in 1 2 4; do
  SVAE_DKW_WK=$wk timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-fp32 > gpurun_out/d3_b.log 2>&1 || exit 1
  echo "WK=$wk $(tail -1 gpurun_out/d3_b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["elbo_per_img"])')"
done; done
for wk in 1 2; do
SVAE_DKW_WK=$wk timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/d3_prof$wk -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-fp32 > gpurun_out/d3_prof.log 2>&1 || exit 1
python3 tools/prof_shapes.py gpurun_out/d3_prof$wk/run_results.db "dense_kw|splitk" > gpurun_out/d3_shapes$wk.txt
done
