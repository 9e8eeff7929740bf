cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for d in bf16x6 bf16; do
  timeout -k 10 120 python tools/diag_grads.py tiny $d || exit 1
done
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
SVAE_KW_BRING=3 SVAE_KW_VEC=1 SVAE_BN_W8=1 timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_golden_gpu.py tests/test_headline_gpu.py -x -q -s --timeout 500 --timeout-method thread > gpurun_out/r04_ring_tests.txt 2>&1 || { tail -30 gpurun_out/r04_ring_tests.txt; exit 1; }
tail -1 gpurun_out/r04_ring_tests.txt
grep -A12 "headline CelebA" gpurun_out/r04_ring_tests.txt | grep -E "bf16x6|gradient"
bash tools/gpu/r04_ab.sh SVAE_KW_BRING=1 SVAE_KW_BRING=3 SVAE_KW_VEC=1,SVAE_BN_W8=1 SVAE_KW_VEC=1,SVAE_BN_W8=1@ab/wt.so SVAE_KW_VEC=1,SVAE_BN_W8=1,SVAE_KW_BRING=1@ab/wt.so
