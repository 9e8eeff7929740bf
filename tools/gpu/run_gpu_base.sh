#!/bin/bash
# baseline: full GPU suite, smoke, kernel-trace DB + per-launch view, bench, host enqueue rate
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1
rc=$?; echo tests_rc=$rc >> gpurun_out/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bf16 -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/prof.log 2>&1 || exit 1
db=$(find gpurun_out/prof_bf16 -name '*.db' | head -n 1)
python tools/prof_launches.py "$db" 1 > gpurun_out/launches.txt 2>&1
python tools/prof_summary.py "$db" > gpurun_out/kernel_stats.txt 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || exit 1
[ "$1" = "host" ] && timeout -k 10 300 python tools/host_rate.py > gpurun_out/host.log 2>&1
exit 0
