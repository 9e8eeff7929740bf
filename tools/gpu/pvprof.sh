#!/bin/bash
# c_pixelvae kernel statistics of the tree (tools/gpu/prof.sh stats)
cd $GRAFT_REPO_ROOT
bash tools/gpu/prof.sh $1 stats --config c_pixelvae --steps 4 --warmup 2
