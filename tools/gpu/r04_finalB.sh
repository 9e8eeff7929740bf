#!/bin/bash
# round-4 check, part B: kernel-trace stats and stream breakdowns, PMC traffic (FETCH_SIZE / WRITE_SIZE
# passes) of the CelebA bf16 / bf16x6, LSUN and c_pixelvae bench commands
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r04_final}
prof() {  # name, bench args
  local n=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_p_$n -o run -- python3 bench.py "$@" > gpurun_out/${TAG}_p_$n.log 2>&1 || return 1
  python3 tools/prof_summary.py gpurun_out/${TAG}_p_$n/run_results.db > gpurun_out/${TAG}_${n}_kernel_stats.txt 2>&1 || true
  python3 tools/stream_breakdown.py gpurun_out/${TAG}_p_$n/run_results.db 28 6 4 > gpurun_out/${TAG}_${n}_streams.txt 2>&1 || true
  rm -rf gpurun_out/${TAG}_p_$n
}
pmc() {  # name, bench args
  local n=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_f_$n -o run -- python3 bench.py "$@" > gpurun_out/${TAG}_f_$n.log 2>&1 || return 1
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${TAG}_w_$n -o run -- python3 bench.py "$@" > gpurun_out/${TAG}_w_$n.log 2>&1 || return 1
  python3 tools/pmc_traffic.py gpurun_out/${TAG}_f_$n gpurun_out/${TAG}_w_$n gpurun_out/${TAG}_${n}pmc_traffic.json $TAG-$n > gpurun_out/${TAG}_${n}pmc.txt
  rm -rf gpurun_out/${TAG}_f_$n gpurun_out/${TAG}_w_$n
}
Q="--no-cpu-baseline --no-fp32"
prof bf16 --steps 10 --warmup 3 $Q || exit 1
head -8 gpurun_out/${TAG}_bf16_streams.txt
prof x6 --dtype bf16x6 --steps 6 --warmup 2 $Q || exit 1
prof lsun --config lsun --steps 6 --warmup 2 $Q || exit 1
prof pv --config c_pixelvae --steps 3 --warmup 1 $Q || exit 1
pmc "" --steps 2 --warmup 1 $Q || exit 1
pmc x6_ --dtype bf16x6 --steps 2 --warmup 1 $Q || exit 1
pmc lsun_ --config lsun --steps 2 --warmup 1 $Q || exit 1
pmc pv_ --config c_pixelvae --steps 1 --warmup 1 $Q || exit 1
ls gpurun_out | grep ${TAG}
