cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/r05_e5.txt
echo "== bf16x6" > $O
timeout -k 10 300 python tools/bench_split.py >> $O 2>&1 || exit 1
echo "== h16" >> $O
timeout -k 10 300 python tools/bench_split.py --h16 --check >> $O 2>&1 || exit 1
grep -v amdgpu.ids $O
