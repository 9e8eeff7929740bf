cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && timeout -k 10 300 python -u tools/graph_probe.py --steps 30 > gpurun_out/graph_probe.log 2>&1; tail -5 gpurun_out/graph_probe.log
