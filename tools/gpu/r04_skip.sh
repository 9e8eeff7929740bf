cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
SVAE_KW_PERSIST_SPLIT=1 timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -q -k bf16x6 --timeout 300 --timeout-method thread > gpurun_out/r04_pst_tests.txt 2>&1 || { tail -30 gpurun_out/r04_pst_tests.txt; exit 1; }
tail -1 gpurun_out/r04_pst_tests.txt
# upper bound of the BN fold: the step without the passes it would remove (results wrong, timing only)
ROUNDS=2 bash tools/gpu/r04_ab.sh SVAE_DBG_SKIP=1 SVAE_DBG_SKIP=2 SVAE_DBG_SKIP=3 SVAE_KW_PERSIST_SPLIT=1 SVAE_KW_PERSIST_SPLIT=2
