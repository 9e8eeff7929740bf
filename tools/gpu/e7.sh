cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/bench_split.py --h16 --check > gpurun_out/r05_e7.txt 2>&1 || { tail -20 gpurun_out/r05_e7.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r05_e7.txt | tail -3
bash tools/gpu/quick.sh r05_q2
