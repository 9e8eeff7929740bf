#!/bin/bash
# Round-6 iteration on the GPU box: GPU suite (optional), one bench line, the split-gather microbench of the
# default library and of variant builds, and an interleaved same-box bench A/B of those variants.
#   SUITE=1 tools/gpu/r06.sh TAG [variant.so ...]
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; shift
if [ "${SUITE:-0}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.txt 2>&1; rc=$?
  tail -2 gpurun_out/${TAG}_gpu_tests.txt
  [ $rc -ne 0 ] && { grep -E "^E |FAILED|Error" gpurun_out/${TAG}_gpu_tests.txt | head -20; exit 1; }
fi
if [ -n "${TESTS}" ]; then
  timeout -k 10 900 python -u -m pytest ${TESTS} -m gpu -x -v -s --timeout 400 --timeout-method thread > gpurun_out/${TAG}_tests.txt 2>&1; rc=$?
  tail -2 gpurun_out/${TAG}_tests.txt
  [ $rc -ne 0 ] && { grep -E "^E |FAILED|Error" gpurun_out/${TAG}_tests.txt | head -20; exit 1; }
fi
timeout -k 10 600 python bench.py --no-cpu-baseline --no-fp32-mode > gpurun_out/${TAG}_bench.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log > gpurun_out/${TAG}_bench.json
python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_bench.json')); print('value', d['value'], d['dtype'], 'ms', d['ms_per_step'], 'bf16', d.get('bf16_value'), 'frac', d['roofline']['frac'], 'elbo', d['elbo_per_img'], 'extra warmup', d.get('warmup_extra_steps'))"
if [ $# -gt 0 ]; then
  BSARGS="--h16 ${MICRO_ARGS}" bash tools/gpu/micro.sh ${TAG}_micro "$@" || exit 1
  specs=()
  for v in "$@"; do specs+=("X=0@$v"); done
  ROUNDS=${ROUNDS:-2} STEPS=30 bash tools/gpu/ab.sh "X=0@sequential-variational-autoencoder_amd/libsvae_hip.so" "${specs[@]}" || exit 1
fi
exit 0
