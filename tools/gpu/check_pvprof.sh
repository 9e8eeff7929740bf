#!/bin/bash
# the round-end check of the tree, then the c_pixelvae kernel statistics (tools/gpu/check.sh, prof.sh)
cd $GRAFT_REPO_ROOT
bash tools/gpu/check.sh $1 && bash tools/gpu/prof.sh $2 stats --config c_pixelvae --steps 4 --warmup 2
