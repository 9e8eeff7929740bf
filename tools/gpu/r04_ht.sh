#!/bin/bash
# wide heads with 16-byte LDS reads in the inner loops: check, then LSUN A/B against the previous build
# (abl/pre_ht.so; same elbo = bitwise)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_heads_gpu.py -x -q -s --timeout 350 --timeout-method thread > gpurun_out/r04_ht_test.txt 2>&1 || { tail -30 gpurun_out/r04_ht_test.txt; exit 1; }
grep "wide heads\|passed" gpurun_out/r04_ht_test.txt
for i in 1 2; do
for spec in "X=0" "SVAE_LIB=$PWD/abl/pre_ht.so"; do
env $spec timeout -k 10 300 python bench.py --config lsun --steps 10 --warmup 3 --no-cpu-baseline --no-fp32-mode --parity-steps 6 > gpurun_out/ht_b.log 2>&1 || { tail -20 gpurun_out/ht_b.log; exit 1; }
echo "${spec##*/}: $(tail -1 gpurun_out/ht_b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("lsun bf16 %.0f img/s %.3f ms | bf16x6 %.0f img/s | elbo %s" % (d["value"], d["ms_per_step"], d["parity_value"], d["elbo_per_img"]))')"
done
done
