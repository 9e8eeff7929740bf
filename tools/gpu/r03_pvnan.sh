#!/bin/bash
# which change makes c_pixelvae training non-finite: the halo conv (SVAE_PC3=0 turns it off) or the init moments
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 0 1; do
  SVAE_PC3=$v timeout -k 10 300 python -u -m pytest tests/test_pixelvae_gpu.py -x -q -k train_and_generate --timeout 200 --timeout-method thread > gpurun_out/pvnan_$v.txt 2>&1; rc=$?
  echo "SVAE_PC3=$v rc=$rc"; tail -1 gpurun_out/pvnan_$v.txt
  case $rc in 124|134|137|139) exit 1;; esac
done
exit 0
