cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/r05_e1.txt
echo "== default" > $O
timeout -k 10 300 python tools/bench_split.py --check >> $O 2>&1 || exit 1
for v in bl1 nosplit; do
  echo "== $v" >> $O
  SVAE_LIB=$PWD/expt/$v.so timeout -k 10 300 python tools/bench_split.py >> $O 2>&1 || exit 1
done
cat $O
