#!/bin/bash
# c_pixelvae: the head's parity suites on the shipping library, then an interleaved bench A/B of a knob
# (knob build with $1=$2 against the shipping library)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_pcconv_gpu.py tests/test_pixelvae_gpu.py tests/test_pcnn_gpu.py -m gpu -x -q -s --timeout 400 --timeout-method thread > gpurun_out/pv_ab_tests.txt 2>&1 || { grep -E "^E |FAILED|Error" gpurun_out/pv_ab_tests.txt | head -20; exit 1; }
tail -1 gpurun_out/pv_ab_tests.txt
grep -E "split head" gpurun_out/pv_ab_tests.txt
K=$PWD/sequential-variational-autoencoder_amd/libsvae_hip_knobs.so
D=$PWD/sequential-variational-autoencoder_amd/libsvae_hip.so
for i in 1 2; do
  for spec in "$1=$2@$K" "X=0@$D"; do
    envs=${spec%@*}; lib=${spec#*@}
    env $envs SVAE_LIB=$lib timeout -k 10 300 python bench.py --config c_pixelvae --steps 6 --warmup 2 --no-secondary --no-cpu-baseline > gpurun_out/pv_ab_b.log 2>&1 || { tail -5 gpurun_out/pv_ab_b.log; exit 1; }
    echo "$envs $(basename $lib): $(tail -1 gpurun_out/pv_ab_b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.1f img/s %.1f ms elbo %s conv %.1f us" % (d["value"], d["ms_per_step"], d["elbo_per_img"], d["roofline"]["avg_conv_us"]))')"
  done
done
