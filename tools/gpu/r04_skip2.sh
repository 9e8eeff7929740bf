cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
# where the backward's critical path is: the step without the side stream's weight-GEMMs / Adam (timing only)
ROUNDS=2 bash tools/gpu/r04_ab.sh SVAE_DBG_SKIP=4 SVAE_DBG_SKIP=8 SVAE_DBG_SKIP=6 SVAE_DBG_SKIP=12
