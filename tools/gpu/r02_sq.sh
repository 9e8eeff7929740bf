#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA --output-format csv -d gpurun_out/r02_sq1 -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-fp32 > gpurun_out/r02_sq1.log 2>&1 || exit 1
python3 tools/sq_summary.py gpurun_out/r02_sq1 > gpurun_out/r02_sq1.txt
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS --output-format csv -d gpurun_out/r02_sq2 -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-fp32 > gpurun_out/r02_sq2.log 2>&1 || exit 1
python3 tools/sq_summary.py gpurun_out/r02_sq2 > gpurun_out/r02_sq2.txt
head -22 gpurun_out/r02_sq1.txt; head -22 gpurun_out/r02_sq2.txt
