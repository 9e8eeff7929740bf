#!/bin/bash
# SQ counters of the bf16x6 and bf16 steps (wave cycles, waits, instruction mix, LDS) -- per-kernel summary
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r04_sq}
for m in bf16x6 bf16; do
CMD="python3 bench.py --dtype $m --steps 2 --warmup 1 --no-cpu-baseline --no-fp32"
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA --output-format csv -d gpurun_out/${TAG}_sq1 -o run -- $CMD > gpurun_out/${TAG}_sq1.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d gpurun_out/${TAG}_sq2 -o run -- $CMD > gpurun_out/${TAG}_sq2.log 2>&1 || exit 1
echo "== $m" >> gpurun_out/${TAG}.txt
python3 tools/sq_summary.py gpurun_out/${TAG}_sq1 >> gpurun_out/${TAG}.txt
python3 tools/sq_summary.py gpurun_out/${TAG}_sq2 >> gpurun_out/${TAG}.txt
rm -rf gpurun_out/${TAG}_sq1 gpurun_out/${TAG}_sq2
done
head -30 gpurun_out/${TAG}.txt
