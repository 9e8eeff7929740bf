#!/bin/bash
# round-end style check: the full GPU suite, smoke(), the default bench line
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r02_full}
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.txt 2>&1; rc=$?
tail -3 gpurun_out/${TAG}_gpu_tests.txt
[ $rc -ne 0 ] && { grep -E "^E |FAILED|Error" gpurun_out/${TAG}_gpu_tests.txt | head -20; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.txt 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.txt; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.txt
timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.json.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench.json.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.json.log > gpurun_out/${TAG}_bench.json
cat gpurun_out/${TAG}_bench.json
