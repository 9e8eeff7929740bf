#!/bin/bash
# HIP API host-time summary of the training step (no counters)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --hip-trace --stats --output-format csv -d gpurun_out/hipt -o run -- python3 tools/host_enqueue.py 10 > gpurun_out/hipt.log 2>&1 || { tail -5 gpurun_out/hipt.log; exit 1; }
grep "host enqueue" gpurun_out/hipt.log
find gpurun_out/hipt -name "*stats*" | head
find gpurun_out/hipt -type f | head -20; for f in $(find gpurun_out/hipt -name "*stats*.csv"); do cp $f gpurun_out/; done
rm -rf gpurun_out/hipt
ls gpurun_out/*stats*.csv
