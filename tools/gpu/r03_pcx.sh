#!/bin/bash
# PixelCNN conv / wgrad parity and per-shape timing, c_pixelvae bench leg
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r03_pcx}
timeout -k 10 300 python -u -m pytest tests/test_pcconv_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.txt 2>&1; rc=$?
tail -1 gpurun_out/${TAG}_tests.txt
[ $rc -ne 0 ] && { grep -E "^E |Error|assert" gpurun_out/${TAG}_tests.txt | head -30; exit 1; }
timeout -k 10 200 python tools/bench_pcconv.py --xb --reps 5 > gpurun_out/${TAG}_cbench.txt 2>&1 || { tail -5 gpurun_out/${TAG}_cbench.txt; exit 1; }
timeout -k 10 200 python tools/bench_pcconv.py --xb --wgrad --reps 5 > gpurun_out/${TAG}_wbench.txt 2>&1 || { tail -5 gpurun_out/${TAG}_wbench.txt; exit 1; }
paste gpurun_out/${TAG}_cbench.txt gpurun_out/${TAG}_wbench.txt | grep -v amdgpu | cut -c1-170
timeout -k 10 600 python bench.py --config c_pixelvae --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_pvae_bench.log 2>&1 || { tail -20 gpurun_out/${TAG}_pvae_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_pvae_bench.log | cut -c1-250
exit 0
