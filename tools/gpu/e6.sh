cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/r05_e6.txt
K=$PWD/sequential-variational-autoencoder_amd/libsvae_hip_knobs.so
echo "== stamps" > $O
SVAE_LIB=$PWD/expt/stamps.so timeout -k 10 300 python tools/bench_split.py --h16 --stamps dec.s1.32,dec.s1.8,d:dec.s1.16 >> $O 2>&1 || exit 1
echo "== knobs default" >> $O
SVAE_LIB=$K timeout -k 10 300 python tools/bench_split.py --h16 >> $O 2>&1 || exit 1
echo "== bm128" >> $O
SVAE_KW_SPLIT_BM=128 SVAE_LIB=$K timeout -k 10 300 python tools/bench_split.py --h16 >> $O 2>&1 || exit 1
echo "== vec" >> $O
SVAE_KW_VEC=1 SVAE_LIB=$K timeout -k 10 300 python tools/bench_split.py --h16 >> $O 2>&1 || exit 1
grep -v amdgpu.ids $O | grep -v "^[a-z:.0-9>]* *(" 
