#!/bin/bash
# iteration: full GPU suite + profile + bench, then SQ counters
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu/run_gpu.sh || exit 1
bash tools/gpu/run_gpu_sq.sh
