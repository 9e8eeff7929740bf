cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
SVAE_LIB=$PWD/expt/stamps.so timeout -k 10 300 python tools/bench_split.py --stamps dec.s1.32,d:dec.s1.32,dec.s1.16,dec.s1.8,dec.s2.8\>16,enc.a.16\>8,rec.b.16 > gpurun_out/r05_e2.txt 2>&1 || exit 1
cat gpurun_out/r05_e2.txt
