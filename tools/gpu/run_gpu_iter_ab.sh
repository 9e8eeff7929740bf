#!/bin/bash
# iteration + same-box A/B of an env switch: run_gpu_iter_ab.sh VAR A B
cd $GRAFT_REPO_ROOT
bash tools/gpu/run_gpu_iter.sh || exit 1
bash tools/gpu/run_gpu_ab.sh "$@"
