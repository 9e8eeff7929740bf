#!/bin/bash
# split-latent FC backward with z through scalar loads (no LDS copy): A/B against the previous build
# (abl/pre_sfb.so; same elbo = bitwise), LSUN and CelebA
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
for spec in "X=0" "SVAE_LIB=$PWD/abl/pre_sfb.so"; do
for cfg in lsun celeba; do
env $spec timeout -k 10 300 python bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline --no-fp32-mode --parity-steps 6 > gpurun_out/sfb_b.log 2>&1 || { tail -20 gpurun_out/sfb_b.log; exit 1; }
echo "${spec##*/} $cfg: $(tail -1 gpurun_out/sfb_b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("bf16 %.0f img/s %.3f ms | bf16x6 %.0f img/s | elbo %s" % (d["value"], d["ms_per_step"], d["parity_value"], d["elbo_per_img"]))')"
done
done
done
