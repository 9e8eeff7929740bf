#!/bin/bash
# Profiles of one bench command on the GPU box (run through gpurun):
#   tools/gpu/prof.sh TAG WHAT [bench args...]
# WHAT (comma-separated):
#   stats   rocprofv3 --kernel-trace --stats: per-kernel summary, per-stream breakdown, per-shape summary
#   pmc     FETCH_SIZE and WRITE_SIZE in separate --pmc passes -> <TAG>_pmc_traffic.json
#   sq      two SQ counter passes (instruction mix / waits; LDS conflicts / memory instructions)
# Outputs go to gpurun_out/<TAG>_*; raw databases are removed after summarising.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; WHAT=$2; shift 2
ARGS=("$@")
[ ${#ARGS[@]} -eq 0 ] && ARGS=(--steps 6 --warmup 2)
Q="--no-cpu-baseline --no-fp32-mode --no-secondary"
if [[ ",$WHAT," == *",stats,"* ]]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_p -o run -- python3 bench.py "${ARGS[@]}" $Q > gpurun_out/${TAG}_p.log 2>&1 || { tail -20 gpurun_out/${TAG}_p.log; exit 1; }
  python3 tools/prof_summary.py gpurun_out/${TAG}_p/run_results.db > gpurun_out/${TAG}_kernel_stats.txt 2>&1
  python3 tools/stream_breakdown.py gpurun_out/${TAG}_p/run_results.db 28 6 4 > gpurun_out/${TAG}_streams.txt 2>&1
  python3 tools/prof_shapes.py gpurun_out/${TAG}_p/run_results.db > gpurun_out/${TAG}_shapes.txt 2>&1
  tail -1 gpurun_out/${TAG}_p.log > gpurun_out/${TAG}_prof_bench.json
  rm -rf gpurun_out/${TAG}_p
  head -12 gpurun_out/${TAG}_streams.txt
fi
if [[ ",$WHAT," == *",pmc,"* ]]; then
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_f -o run -- python3 bench.py "${ARGS[@]}" $Q > gpurun_out/${TAG}_f.log 2>&1 || { tail -20 gpurun_out/${TAG}_f.log; exit 1; }
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${TAG}_w -o run -- python3 bench.py "${ARGS[@]}" $Q > gpurun_out/${TAG}_w.log 2>&1 || { tail -20 gpurun_out/${TAG}_w.log; exit 1; }
  python3 tools/pmc_traffic.py gpurun_out/${TAG}_f gpurun_out/${TAG}_w gpurun_out/${TAG}_pmc_traffic.json $TAG > gpurun_out/${TAG}_pmc.txt
  rm -rf gpurun_out/${TAG}_f gpurun_out/${TAG}_w
  head -20 gpurun_out/${TAG}_pmc.txt
fi
if [[ ",$WHAT," == *",sq,"* ]]; then
  timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA --output-format csv -d gpurun_out/${TAG}_sq1 -o run -- python3 bench.py "${ARGS[@]}" $Q > gpurun_out/${TAG}_sq1.log 2>&1 || { tail -20 gpurun_out/${TAG}_sq1.log; exit 1; }
  timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d gpurun_out/${TAG}_sq2 -o run -- python3 bench.py "${ARGS[@]}" $Q > gpurun_out/${TAG}_sq2.log 2>&1 || { tail -20 gpurun_out/${TAG}_sq2.log; exit 1; }
  python3 tools/sq_summary.py gpurun_out/${TAG}_sq1 > gpurun_out/${TAG}_sq.txt
  python3 tools/sq_summary.py gpurun_out/${TAG}_sq2 >> gpurun_out/${TAG}_sq.txt
  rm -rf gpurun_out/${TAG}_sq1 gpurun_out/${TAG}_sq2
  head -12 gpurun_out/${TAG}_sq.txt
fi
exit 0
