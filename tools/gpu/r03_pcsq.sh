#!/bin/bash
# SQ counters of the halo PixelCNN conv on its largest shape (64x64, 160 -> 160, [2, 3], bf16 input)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r03_pcsq}
CMD="python3 tools/bench_pcconv.py --xb --shape 64,160,160,2,3,0 --reps 3"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA --output-format csv -d gpurun_out/${TAG}_sq1 -o run -- $CMD > gpurun_out/${TAG}_sq1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS --output-format csv -d gpurun_out/${TAG}_sq2 -o run -- $CMD > gpurun_out/${TAG}_sq2.log 2>&1 || exit 1
python3 tools/sq_summary.py gpurun_out/${TAG}_sq1 > gpurun_out/${TAG}.txt
python3 tools/sq_summary.py gpurun_out/${TAG}_sq2 >> gpurun_out/${TAG}.txt
rm -rf gpurun_out/${TAG}_sq1 gpurun_out/${TAG}_sq2
cat gpurun_out/${TAG}.txt
