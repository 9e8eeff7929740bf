#!/bin/bash
# same-box A/B of the split / tile-fill knobs on the current schedule, two interleaved rounds
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/knobs
for rep in 1 2; do
  for cfg in "base" "SVAE_WH_TARGET=384" "SVAE_WH_TARGET=512" "SVAE_WH_TARGET=192" "SVAE_WH_MINCH=6" "SVAE_WH_MINCH=12" "SVAE_HALO_FILL=384" "SVAE_HALO_FILL=768"; do
    if [ "$cfg" = base ]; then envs=(); else envs=("$cfg"); fi
    env "${envs[@]}" timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/knobs/run.json 2>/dev/null || exit 1
    python -c "import json,sys;d=json.load(open('gpurun_out/knobs/run.json'));print(sys.argv[1],sys.argv[2],d['ms_per_step'],d['value'])" "$rep" "$cfg" | tee -a gpurun_out/knobs/summary.txt
  done
done
