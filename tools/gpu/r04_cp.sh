cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_engine_gpu.py tests/test_wgrad_bf16_gpu.py -x -q -k "bf16x6 or split" --timeout 300 --timeout-method thread > gpurun_out/r04_cp_tests.txt 2>&1 || { tail -30 gpurun_out/r04_cp_tests.txt; exit 1; }
tail -1 gpurun_out/r04_cp_tests.txt
ROUNDS=2 bash tools/gpu/r04_ab.sh SVAE_WH2_SPLIT_CP=256
