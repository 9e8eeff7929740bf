#!/bin/bash
# split-bf16 (bf16x6) mode: FETCH_SIZE calibration, parity suites in both fp32-class modes, the
# headline printout, chain-variant bounds, and the bench line with parity_value
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r03_v1}
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_calib -o run -- ./tools/calib/fetch_calib > gpurun_out/${TAG}_calib.log 2>&1 || { tail -5 gpurun_out/${TAG}_calib.log; exit 1; }
python3 tools/calib/fetch_calib.py gpurun_out/${TAG}_calib > gpurun_out/${TAG}_fetch_calib.txt; cat gpurun_out/${TAG}_fetch_calib.txt; rm -rf gpurun_out/${TAG}_calib
timeout -k 10 900 python -u -m pytest tests/test_engine_gpu.py tests/test_golden_gpu.py tests/test_checkpoint_gpu.py tests/test_generate_gpu.py tests/test_chain_variants_gpu.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.txt 2>&1; rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/${TAG}_tests.txt | tail -8
[ $rc -ne 0 ] && { grep -E "^E " gpurun_out/${TAG}_tests.txt | head -20; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_headline_gpu.py -x -v -s --timeout 550 --timeout-method thread > gpurun_out/${TAG}_headline.txt 2>&1; rc=$?
grep -A14 "headline CelebA" gpurun_out/${TAG}_headline.txt
[ $rc -ne 0 ] && { grep -E "^E " gpurun_out/${TAG}_headline.txt | head -20; exit 1; }
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log
