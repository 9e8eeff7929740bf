#!/bin/bash
# c_pixelvae on the GPU box: the head / chain parity tests, then the bench line (optionally an A/B of the knob
# build with and without a switch: PV_AB="ENV=V").
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1
timeout -k 10 700 python -u -m pytest tests/test_pcconv_gpu.py tests/test_pcnn_gpu.py tests/test_pixelvae_gpu.py -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/${TAG}_tests.txt 2>&1 || { tail -30 gpurun_out/${TAG}_tests.txt; exit 1; }
tail -1 gpurun_out/${TAG}_tests.txt
timeout -k 10 600 python bench.py --config c_pixelvae --steps 5 --warmup 2 > gpurun_out/${TAG}_bench.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log > gpurun_out/${TAG}_pixelvae_bench.json
python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_pixelvae_bench.json')); print('value', d['value'], d['dtype'], 'ms', d['ms_per_step'], 'parity', d.get('parity_value'), 'cpu', d.get('cpu_baseline', {}).get('value'), 'frac', d['roofline']['frac'])"
exit 0
