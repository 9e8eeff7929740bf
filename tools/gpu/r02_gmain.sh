#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/bench_gather.py main 2 > gpurun_out/gmain.log 2>&1 || { tail -20 gpurun_out/gmain.log; exit 1; }
cat gpurun_out/gmain.log
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/gmain_prof -o run -- python3 tools/bench_gather.py main 2 > gpurun_out/gmain_p.log 2>&1 || exit 1
python3 tools/prof_shapes.py gpurun_out/gmain_prof/run_results.db "halo|igemm|splitk"
