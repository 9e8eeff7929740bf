#!/bin/bash
# SQ counters of the isolated weight-GEMM shapes (tools/bench_wgrad.py step storage)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA --output-format csv -d gpurun_out/wsq1 -o run -- python3 tools/bench_wgrad.py 5 2 step > gpurun_out/wsq1.log 2>&1 || exit 1
python3 tools/sq_summary.py gpurun_out/wsq1 > gpurun_out/wsq1.txt
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d gpurun_out/wsq2 -o run -- python3 tools/bench_wgrad.py 5 2 step > gpurun_out/wsq2.log 2>&1 || exit 1
python3 tools/sq_summary.py gpurun_out/wsq2 > gpurun_out/wsq2.txt
rm -rf gpurun_out/wsq1 gpurun_out/wsq2
cat gpurun_out/wsq1.txt gpurun_out/wsq2.txt
