#!/bin/bash
# round-4 check, part A: GPU suite, headline / c_pixelvae printouts, smoke, bench lines (CelebA with the
# CPU baseline and the parity mode, LSUN with its own CPU baseline and parity leg, c_pixelvae), the
# dependent-launch boundary calibration
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r04_final}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.txt 2>&1; rc=$?
tail -2 gpurun_out/${TAG}_gpu_tests.txt
[ $rc -ne 0 ] && { grep -E "^E |FAILED|Error" gpurun_out/${TAG}_gpu_tests.txt | head -20; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_headline_gpu.py tests/test_pixelvae_gpu.py tests/test_dp8_gpu.py -x -v -s --timeout 550 --timeout-method thread > gpurun_out/${TAG}_headline.txt 2>&1 || { tail -30 gpurun_out/${TAG}_headline.txt; exit 1; }
grep -A16 "headline CelebA" gpurun_out/${TAG}_headline.txt | head -20
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.txt 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.txt; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.txt
timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.json.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench.json.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.json.log > gpurun_out/${TAG}_bench.json
cat gpurun_out/${TAG}_bench.json
timeout -k 10 600 python bench.py --config lsun --no-fp32-mode > gpurun_out/${TAG}_lsun_bench.json.log 2>&1 || { tail -20 gpurun_out/${TAG}_lsun_bench.json.log; exit 1; }
tail -1 gpurun_out/${TAG}_lsun_bench.json.log > gpurun_out/${TAG}_lsun_bench.json
timeout -k 10 600 python bench.py --config c_pixelvae --steps 10 --warmup 3 > gpurun_out/${TAG}_pixelvae_bench.json.log 2>&1 || { tail -20 gpurun_out/${TAG}_pixelvae_bench.json.log; exit 1; }
tail -1 gpurun_out/${TAG}_pixelvae_bench.json.log > gpurun_out/${TAG}_pixelvae_bench.json
timeout -k 10 120 tools/calib/boundary > gpurun_out/${TAG}_boundary.txt 2>&1 || exit 1
cat gpurun_out/${TAG}_boundary.txt
