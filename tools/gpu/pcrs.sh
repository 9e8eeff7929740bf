#!/bin/bash
# Row-staged fp16-plane conv (pc_conv3r) on the GPU box: its parity tests, then the per-shape microbench of the
# knob build with SVAE_PC_RS=0 (pc_conv3 HP; outputs saved) and =1 (pc_conv3r; compared bitwise), twice.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1
timeout -k 10 400 python -u -m pytest tests/test_pcconv_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "planes" > gpurun_out/${TAG}_tests.txt 2>&1 || { tail -30 gpurun_out/${TAG}_tests.txt; exit 1; }
tail -1 gpurun_out/${TAG}_tests.txt
K=$PWD/sequential-variational-autoencoder_amd/libsvae_hip_knobs.so
for r in 1 2; do
  SVAE_LIB=$K SVAE_PC_RS=0 timeout -k 10 300 python -u tools/bench_pcconv_hp.py --save /tmp/pc_ref.pt > gpurun_out/${TAG}_rs0_$r.txt 2>&1 || { tail -20 gpurun_out/${TAG}_rs0_$r.txt; exit 1; }
  SVAE_LIB=$K SVAE_PC_RS=1 timeout -k 10 300 python -u tools/bench_pcconv_hp.py --compare /tmp/pc_ref.pt > gpurun_out/${TAG}_rs1_$r.txt 2>&1 || { tail -20 gpurun_out/${TAG}_rs1_$r.txt; exit 1; }
done
paste gpurun_out/${TAG}_rs0_2.txt gpurun_out/${TAG}_rs1_2.txt | grep -v amdgpu.ids
exit 0
