#!/bin/bash
# round 2 re-entry: full GPU suite, smoke, bench line, hipGraph probe of the committed tree
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 200 --timeout-method thread > gpurun_out/r02s_tests.log 2>&1
rc=$?; echo tests_rc=$rc; grep -E "passed|failed|error" gpurun_out/r02s_tests.log | tail -5
[ $rc -ne 0 ] && { tail -40 gpurun_out/r02s_tests.log; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02s_smoke.log 2>&1 || { cat gpurun_out/r02s_smoke.log; exit 1; }
tail -1 gpurun_out/r02s_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/r02s_bench.log 2>&1 || { tail -20 gpurun_out/r02s_bench.log; exit 1; }
tail -1 gpurun_out/r02s_bench.log
timeout -k 10 300 python -u tools/graph_probe.py --steps 30 > gpurun_out/r02s_graph.log 2>&1; tail -5 gpurun_out/r02s_graph.log
