#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/host_enqueue.py 30 > gpurun_out/host_enq.log 2>&1 || { tail -5 gpurun_out/host_enq.log; exit 1; }
cat gpurun_out/host_enq.log | grep -v amdgpu.ids
timeout -k 10 300 python tools/host_enqueue.py 30 > gpurun_out/host_enq.log 2>&1 || { tail -5 gpurun_out/host_enq.log; exit 1; }
cat gpurun_out/host_enq.log | grep -v amdgpu.ids
