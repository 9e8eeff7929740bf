#!/bin/bash
# fused-plane weight gradients on the tap-row kernel for every kernel width (SVAE_PW4_ALLKW): the head's
# plane tests on that path, then the c_pixelvae A/B
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
K=$PWD/sequential-variational-autoencoder_amd/libsvae_hip_knobs.so
SVAE_LIB=$K SVAE_PW4_ALLKW=1 timeout -k 10 600 python -u -m pytest tests/test_pcconv_gpu.py tests/test_pixelvae_gpu.py -k "planes or split_head" -m gpu -x -q -s --timeout 300 --timeout-method thread > gpurun_out/pw4_tests.txt 2>&1 || { grep -E "^E |FAILED|Error" gpurun_out/pw4_tests.txt | head; exit 1; }
tail -1 gpurun_out/pw4_tests.txt; grep "split head" gpurun_out/pw4_tests.txt
D=$PWD/sequential-variational-autoencoder_amd/libsvae_hip.so
for i in 1 2; do
  for spec in "SVAE_PW4_ALLKW=1@$K" "X=0@$D"; do
    envs=${spec%@*}; lib=${spec#*@}
    env $envs SVAE_LIB=$lib timeout -k 10 300 python bench.py --config c_pixelvae --steps 6 --warmup 2 --no-secondary --no-cpu-baseline > gpurun_out/pv_ab_b.log 2>&1 || { tail -5 gpurun_out/pv_ab_b.log; exit 1; }
    echo "$envs $(basename $lib): $(tail -1 gpurun_out/pv_ab_b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.1f img/s %.1f ms elbo %s" % (d["value"], d["ms_per_step"], d["elbo_per_img"]))')"
  done
done
