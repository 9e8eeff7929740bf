#!/bin/bash
cd $GRAFT_REPO_ROOT
bash tools/gpu/prof.sh r05_g6 stats,pmc,sq && bash tools/gpu/prof.sh r05_gbf stats,pmc,sq --dtype bf16 --steps 6 --warmup 2 && bash tools/gpu/prof.sh r05_gpv stats,pmc --config c_pixelvae --steps 2 --warmup 1
