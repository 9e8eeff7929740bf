#!/bin/bash
# round-end check of the committed tree: GPU suite, headline / c_pixelvae printouts, smoke, PMC traffic
# passes of the bench command, the c_pixelvae bench leg,
# the default bench line (reading that traffic), kernel-trace stats and the stream breakdown
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r03_final}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.txt 2>&1; rc=$?
tail -2 gpurun_out/${TAG}_gpu_tests.txt
[ $rc -ne 0 ] && { grep -E "^E |FAILED|Error" gpurun_out/${TAG}_gpu_tests.txt | head -20; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_headline_gpu.py tests/test_pixelvae_gpu.py -x -v -s --timeout 550 --timeout-method thread > gpurun_out/${TAG}_headline.txt 2>&1 || { tail -30 gpurun_out/${TAG}_headline.txt; exit 1; }
grep -A14 "headline CelebA" gpurun_out/${TAG}_headline.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.txt 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.txt; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.txt
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_pmc_fetch -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-fp32 > gpurun_out/${TAG}_pmc_fetch.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${TAG}_pmc_write -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-fp32 > gpurun_out/${TAG}_pmc_write.log 2>&1 || exit 1
python3 tools/pmc_traffic.py gpurun_out/${TAG}_pmc_fetch gpurun_out/${TAG}_pmc_write gpurun_out/${TAG}_pmc_traffic.json $TAG > gpurun_out/${TAG}_pmc.txt; rm -rf gpurun_out/${TAG}_pmc_fetch gpurun_out/${TAG}_pmc_write
cp gpurun_out/${TAG}_pmc_traffic.json profiles/
timeout -k 10 600 python bench.py --config c_pixelvae --steps 10 --warmup 3 > gpurun_out/${TAG}_pixelvae_bench.json.log 2>&1 || { tail -20 gpurun_out/${TAG}_pixelvae_bench.json.log; exit 1; }
tail -1 gpurun_out/${TAG}_pixelvae_bench.json.log > gpurun_out/${TAG}_pixelvae_bench.json
timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.json.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench.json.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.json.log > gpurun_out/${TAG}_bench.json
cat gpurun_out/${TAG}_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-fp32 > gpurun_out/${TAG}_prof.log 2>&1 || exit 1
python3 tools/prof_summary.py gpurun_out/${TAG}_prof/run_results.db > gpurun_out/${TAG}_kernel_stats.txt 2>&1 || true
python3 tools/stream_breakdown.py gpurun_out/${TAG}_prof/run_results.db 28 20 8 > gpurun_out/${TAG}_streams.txt 2>&1 || true
head -8 gpurun_out/${TAG}_streams.txt
# LSUN-bedroom (BASELINE configs[2], B=256) and the parity mode's kernel stats
timeout -k 10 300 python bench.py --config lsun --steps 10 --warmup 3 --no-cpu-baseline --no-fp32 > gpurun_out/${TAG}_lsun_bench.json.log 2>&1 || { tail -20 gpurun_out/${TAG}_lsun_bench.json.log; exit 1; }
tail -1 gpurun_out/${TAG}_lsun_bench.json.log > gpurun_out/${TAG}_lsun_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof6 -o run -- python3 bench.py --dtype bf16x6 --steps 6 --warmup 2 --no-cpu-baseline --no-fp32 > gpurun_out/${TAG}_prof6.log 2>&1 || exit 1
python3 tools/prof_summary.py gpurun_out/${TAG}_prof6/run_results.db > gpurun_out/${TAG}_bf16x6_kernel_stats.txt 2>&1 || true
python3 tools/stream_breakdown.py gpurun_out/${TAG}_prof6/run_results.db 28 6 4 > gpurun_out/${TAG}_bf16x6_streams.txt 2>&1 || true
rm -rf gpurun_out/${TAG}_prof6
