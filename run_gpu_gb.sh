#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/bench_gather.py > gpurun_out/gb.log 2>&1 || exit 1
rocprofv3 -L > gpurun_out/counters.txt 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d gpurun_out/pmc_gb -o run -- python3 tools/bench_gather.py 1 > gpurun_out/pmc_gb.log 2>&1
echo pmc_rc=$? >> gpurun_out/pmc_gb.log
