cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for d in bf16x6 bf16; do
  timeout -k 10 120 python tools/diag_grads.py tiny $d || exit 1
done
