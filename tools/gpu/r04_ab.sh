#!/bin/bash
# bench A/B (interleaved, ROUNDS rounds) over settings "ENV=V[,ENV2=V2][@lib.so]" ...; the first is the baseline
# prints the bf16 value and the bf16x6 parity_value of each run
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in $(seq 1 ${ROUNDS:-2}); do
  for spec in "X=0" "$@"; do
    envs=${spec%@*}; lib=""
    [[ "$spec" == *@* ]] && lib=$PWD/${spec#*@}
    envs=${envs//,/ }
    env $envs ${lib:+SVAE_LIB=$lib} timeout -k 10 300 python bench.py --steps ${STEPS:-30} --warmup 5 --no-cpu-baseline --no-fp32-mode --parity-steps 20 > gpurun_out/ab_b.log 2>&1 || { tail -20 gpurun_out/ab_b.log; exit 1; }
    echo "$spec: $(tail -1 gpurun_out/ab_b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("bf16 %.0f img/s %.3f ms | bf16x6 %.0f img/s %.3f ms | elbo %s" % (d["value"], d["ms_per_step"], d["parity_value"], d["parity_ms_per_step"], d["elbo_per_img"]))')"
  done
done
