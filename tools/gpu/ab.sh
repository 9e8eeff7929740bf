#!/bin/bash
# Interleaved same-box bench A/B (run through gpurun):
#   ROUNDS=2 STEPS=30 tools/gpu/ab.sh "ENV=V[,ENV2=V2][@lib.so]" ...
# Every setting runs with the -DSVAE_KNOBS build (libsvae_hip_knobs.so, csrc/knobs.h) unless it names its own
# library after '@'; the first run of each round is the knob build with no switch (the baseline).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
K=$PWD/sequential-variational-autoencoder_amd/libsvae_hip_knobs.so
for i in $(seq 1 ${ROUNDS:-2}); do
  for spec in "X=0" "$@"; do
    envs=${spec%@*}; lib=$K
    [[ "$spec" == *@* ]] && lib=$PWD/${spec#*@}
    envs=${envs//,/ }
    env $envs SVAE_LIB=$lib timeout -k 10 300 python bench.py --steps ${STEPS:-30} --warmup 5 --no-cpu-baseline --no-fp32-mode --parity-steps 20 ${BENCH_ARGS} > gpurun_out/ab_b.log 2>&1 || { tail -20 gpurun_out/ab_b.log; exit 1; }
    echo "$spec: $(tail -1 gpurun_out/ab_b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%s %.0f img/s %.3f ms | bf16 %s | elbo %s" % (d["dtype"], d["value"], d["ms_per_step"], d.get("bf16_value"), d["elbo_per_img"]))')"
  done
done
