#!/bin/bash
# quick GPU check: a test subset (TESTS, default the parity suites of the split mode) and one bench line
#   tools/gpu/quick.sh TAG [pytest args...]
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; shift
T=("$@")
[ ${#T[@]} -eq 0 ] && T=(tests/test_engine_gpu.py tests/test_golden_gpu.py tests/test_gather_bf16_gpu.py)
timeout -k 10 900 python -u -m pytest "${T[@]}" -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/${TAG}_tests.txt 2>&1; rc=$?
tail -3 gpurun_out/${TAG}_tests.txt
[ $rc -ne 0 ] && { grep -E "^E |FAILED|Error" gpurun_out/${TAG}_tests.txt | head -30; exit 1; }
timeout -k 10 600 python bench.py --no-cpu-baseline --no-fp32-mode > gpurun_out/${TAG}_bench.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log > gpurun_out/${TAG}_bench.json
python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_bench.json')); print('value', d['value'], d['dtype'], 'ms', d['ms_per_step'], 'bf16', d.get('bf16_value'), 'frac', d['roofline']['frac'], 'elbo', d['elbo_per_img'])"
