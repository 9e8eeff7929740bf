#!/bin/bash
# Split-mode gather microbench (tools/bench_split.py) of the default library and of variant builds:
#   tools/gpu/micro.sh TAG [lib.so ...]     (variant builds: SVAE_CFLAGS=... SVAE_BUILD_OUT=expt/x.so build.py)
# BSARGS passes extra tools/bench_split.py arguments (e.g. "--h16 --check" or "--stamps dec.s1.32").
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; shift
O=gpurun_out/${TAG}.txt
echo "== default" > $O
timeout -k 10 300 python tools/bench_split.py ${BSARGS} >> $O 2>&1 || { tail -20 $O; exit 1; }
for v in "$@"; do
  echo "== $v" >> $O
  SVAE_LIB=$PWD/$v timeout -k 10 300 python tools/bench_split.py ${BSARGS} >> $O 2>&1 || { tail -20 $O; exit 1; }
done
grep -v amdgpu.ids $O | grep -E "^==|per step"
