#!/bin/bash
# round 2, first call: new parity tests, conforming bench line, wgrad microbench + SQ counters
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_headline_gpu.py tests/test_train_api_gpu.py tests/test_checkpoint_gpu.py tests/test_fused_adam_gpu.py > gpurun_out/r02_tests.log 2>&1 || { tail -60 gpurun_out/r02_tests.log; exit 1; }
grep -E "passed|failed|headline|x_hat|gradients|iteration|ELBO" gpurun_out/r02_tests.log | tail -30
timeout -k 10 120 python tools/bench_wgrad.py > gpurun_out/r02_wgrad.log 2>&1 || { cat gpurun_out/r02_wgrad.log; exit 1; }
cat gpurun_out/r02_wgrad.log
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA --output-format csv -d gpurun_out/r02_sq1 -o run -- python3 tools/bench_wgrad.py 3 > gpurun_out/r02_sq1.log 2>&1 || exit 1
timeout -k 10 400 python bench.py > gpurun_out/r02_bench.log 2>&1 || { tail -20 gpurun_out/r02_bench.log; exit 1; }
tail -1 gpurun_out/r02_bench.log
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVES SQ_WAVE_CYCLES SQ_INST_CYCLES_VMEM --output-format csv -d gpurun_out/r02_sq2 -o run -- python3 tools/bench_wgrad.py 3 > gpurun_out/r02_sq2.log 2>&1
python tools/sq_summary.py gpurun_out/r02_sq1 > gpurun_out/r02_sq1.txt 2>&1; cat gpurun_out/r02_sq1.txt
