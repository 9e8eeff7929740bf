#!/bin/bash
# Round-end style check of a committed tree on the GPU box (run through gpurun):
#   tools/gpu/check.sh TAG [suite,headline,smoke,bench,lsun,pixelvae,boundary]   (default: all of them)
# GPU suite, the headline / c_pixelvae / DP8 parity printouts, smoke(), the bench lines (CelebA with the
# CPU baseline and the other-mode legs, LSUN, c_pixelvae) and the dependent-launch boundary calibration.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-check}
WHAT=",${2:-suite,headline,smoke,bench,lsun,pixelvae,boundary},"
if [[ $WHAT == *",suite,"* ]]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.txt 2>&1; rc=$?
  tail -2 gpurun_out/${TAG}_gpu_tests.txt
  [ $rc -ne 0 ] && { grep -E "^E |FAILED|Error" gpurun_out/${TAG}_gpu_tests.txt | head -20; exit 1; }
fi
if [[ $WHAT == *",headline,"* ]]; then
  timeout -k 10 600 python -u -m pytest tests/test_headline_gpu.py tests/test_pixelvae_gpu.py tests/test_dp8_gpu.py -x -v -s --timeout 550 --timeout-method thread > gpurun_out/${TAG}_headline.txt 2>&1 || { tail -30 gpurun_out/${TAG}_headline.txt; exit 1; }
  grep -A16 "headline CelebA" gpurun_out/${TAG}_headline.txt | head -20
fi
if [[ $WHAT == *",smoke,"* ]]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.txt 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.txt; exit 1; }
  tail -1 gpurun_out/${TAG}_smoke.txt
fi
line() {  # name, bench args
  local n=$1; shift
  timeout -k 10 600 python bench.py "$@" > gpurun_out/${TAG}_${n}.json.log 2>&1 || { tail -20 gpurun_out/${TAG}_${n}.json.log; exit 1; }
  tail -1 gpurun_out/${TAG}_${n}.json.log > gpurun_out/${TAG}_${n}.json
  cat gpurun_out/${TAG}_${n}.json
}
[[ $WHAT == *",bench,"* ]] && line bench
[[ $WHAT == *",lsun,"* ]] && line lsun_bench --config lsun --no-fp32-mode
[[ $WHAT == *",pixelvae,"* ]] && line pixelvae_bench --config c_pixelvae --steps 10 --warmup 3
if [[ $WHAT == *",boundary,"* ]]; then
  timeout -k 10 120 tools/calib/boundary > gpurun_out/${TAG}_boundary.txt 2>&1 || exit 1
  cat gpurun_out/${TAG}_boundary.txt
fi
exit 0
