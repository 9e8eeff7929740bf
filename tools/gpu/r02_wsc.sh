#!/bin/bash
# small-Cin weight-GEMM: op-level check vs the generic kernel, GPU suite, bench A/B
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/dpre_bitwise.py celeba 32 ${CMPVAR:-SVAE_NO_WSC=1} > gpurun_out/wsc_cmp.txt 2>&1; echo "cmp rc=$?"; tail -1 gpurun_out/wsc_cmp.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/wsc_gpu_tests.txt 2>&1; rc=$?
tail -2 gpurun_out/wsc_gpu_tests.txt
[ $rc -ne 0 ] && { grep -E "^E |FAILED|Error" gpurun_out/wsc_gpu_tests.txt | head -30; exit 1; }
bash tools/gpu/r02_envab.sh ${CMPVAR:-SVAE_NO_WSC=1}
