cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/r05_e4.txt
echo "== default" > $O
timeout -k 10 300 python tools/bench_split.py >> $O 2>&1 || exit 1
echo "== bm128" >> $O
SVAE_LIB=$PWD/expt/bm128.so timeout -k 10 300 python tools/bench_split.py --check >> $O 2>&1 || exit 1
grep -v amdgpu.ids $O
