#!/bin/bash
# tools/dist_overhead.py in each mode, default hardware queues and 8 (run through gpurun)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/${1:-dist}_overhead.txt
: > $O
for q in default 8; do
  for m in none pg pg_hook; do
    if [ $q = default ]; then timeout -k 10 200 python tools/dist_overhead.py $m >> $O 2>&1 || exit 1
    else GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python tools/dist_overhead.py $m >> $O 2>&1 || exit 1; fi
  done
done
grep ms/step $O
