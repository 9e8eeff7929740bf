#!/bin/bash
# halo PixelCNN weight gradient: parity, per-shape timing (old kernel vs halo), head tests, c_pixelvae bench leg
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r03_pw3}
timeout -k 10 300 python -u -m pytest tests/test_pcconv_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.txt 2>&1; rc=$?
tail -3 gpurun_out/${TAG}_tests.txt
[ $rc -ne 0 ] && { grep -E "^E |Error|assert" gpurun_out/${TAG}_tests.txt | head -30; exit 1; }
for v in 0 1; do
  SVAE_PW3=$v timeout -k 10 200 python tools/bench_pcconv.py --xb --wgrad --reps 5 > gpurun_out/${TAG}_wbench_$v.txt 2>&1 || { tail -5 gpurun_out/${TAG}_wbench_$v.txt; exit 1; }
done
paste gpurun_out/${TAG}_wbench_0.txt gpurun_out/${TAG}_wbench_1.txt | grep -v amdgpu | cut -c1-170
timeout -k 10 600 python -u -m pytest tests/test_pcnn_gpu.py tests/test_pixelvae_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_head_tests.txt 2>&1; rc=$?
tail -2 gpurun_out/${TAG}_head_tests.txt
[ $rc -ne 0 ] && { grep -E "^E |Error" gpurun_out/${TAG}_head_tests.txt | head -20; exit 1; }
timeout -k 10 600 python bench.py --config c_pixelvae --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_pvae_bench.log 2>&1 || { tail -20 gpurun_out/${TAG}_pvae_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_pvae_bench.log | cut -c1-300
exit 0
