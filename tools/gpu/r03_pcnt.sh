#!/bin/bash
# halo conv column-tile width A/B (SVAE_PC3_NT) on the head shapes, then c_pixelvae
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 5 3 2; do
  SVAE_PC3_NT=$v timeout -k 10 200 python tools/bench_pcconv.py --xb --reps 5 > gpurun_out/pcnt_$v.txt 2>&1 || { tail -5 gpurun_out/pcnt_$v.txt; exit 1; }
done
paste gpurun_out/pcnt_5.txt gpurun_out/pcnt_3.txt gpurun_out/pcnt_2.txt | grep -v amdgpu | cut -c1-62,64-114,116-170
for v in 5 2; do
  SVAE_PC3_NT=$v timeout -k 10 600 python bench.py --config c_pixelvae --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/pcnt_b$v.log 2>&1 || { tail -20 gpurun_out/pcnt_b$v.log; exit 1; }
  echo "NT=$v $(tail -1 gpurun_out/pcnt_b$v.log | cut -c1-200)"
done
