#!/bin/bash
# GPU suite then N bench runs (value, ms/step, ELBO)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-chk}
N=${2:-2}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.txt 2>&1; rc=$?
tail -2 gpurun_out/${TAG}_gpu_tests.txt
[ $rc -ne 0 ] && { grep -E "^E |FAILED|Error" gpurun_out/${TAG}_gpu_tests.txt | head -20; exit 1; }
for i in $(seq 1 $N); do
  timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-fp32 > gpurun_out/${TAG}_b.log 2>&1 || { tail -20 gpurun_out/${TAG}_b.log; exit 1; }
  echo "bench $(tail -1 gpurun_out/${TAG}_b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["elbo_per_img"], d["roofline"]["avg_launch_us"])')"
done
