#!/bin/bash
# round 4: the new / changed GPU tests with their printouts (-s), then the default bench line
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r04_new}
timeout -k 10 600 python -u -m pytest tests/test_dp8_gpu.py tests/test_fused_adam_gpu.py tests/test_pixelvae_gpu.py -x -v -s --timeout 400 --timeout-method thread > gpurun_out/${TAG}_tests.txt 2>&1 || { tail -40 gpurun_out/${TAG}_tests.txt; exit 1; }
grep -E "PASS|FAIL|DP8|rank|sequential|init_every|c_pixelvae" gpurun_out/${TAG}_tests.txt | tail -40
timeout -k 10 600 python -u -m pytest tests/test_headline_gpu.py -x -v -s --timeout 550 --timeout-method thread > gpurun_out/${TAG}_headline.txt 2>&1 || { tail -40 gpurun_out/${TAG}_headline.txt; exit 1; }
grep -A16 "headline CelebA" gpurun_out/${TAG}_headline.txt
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench.json.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench.json.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.json.log
