#!/bin/bash
# the c_pixelvae head A/B of one switch (tools/gpu/pv_ab.sh), then the round-end check of the tree (check.sh)
cd $GRAFT_REPO_ROOT
bash tools/gpu/pv_ab.sh $1 $2 && bash tools/gpu/check.sh $3
