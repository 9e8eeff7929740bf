#!/bin/bash
# head tests (conv / wgrad parity, seeded dropout, oracle parity) and the c_pixelvae bench leg
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r03_pcz}
timeout -k 10 600 python -u -m pytest tests/test_pcconv_gpu.py tests/test_pcnn_gpu.py tests/test_pixelvae_gpu.py -x -q -s --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.txt 2>&1; rc=$?
grep -E "passed|failed|seeded dropout|c_pixelvae small" gpurun_out/${TAG}_tests.txt | tail -4
[ $rc -ne 0 ] && { grep -E "^E |Error" gpurun_out/${TAG}_tests.txt | head -20; exit 1; }
timeout -k 10 600 python bench.py --config c_pixelvae --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_pvae_bench.log 2>&1 || { tail -20 gpurun_out/${TAG}_pvae_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_pvae_bench.log | cut -c1-250
exit 0
