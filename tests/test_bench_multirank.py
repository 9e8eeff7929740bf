"""bench.py's N > 1 path: the code the driver's scaling run executes first.

The GPU test runs ``bench.py --gpus 2`` end to end on the one-GPU test box: bench.py spawns two ranks
through torch.distributed.run before any GPU call, both ranks share the GPU, and the process group is
gloo (``--dist-backend gloo``) because RCCL refuses two ranks on one device.  Everything else is the
8-GPU code path: per-rank contiguous shards, the overlapped per-step gradient buckets, the barrier +
synchronize bracket, the MAX-over-ranks elapsed time and the ELBO all-reduce, and rank 0's one JSON
line.  The CPU tests check the argument plumbing: RCCL is the default backend, and a rank without a
GPU of its own is refused under RCCL."""
import importlib.util
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_default_process_group_is_rccl():
    b = _bench()
    args = b.make_parser().parse_args(["--gpus", "8"])
    assert args.dist_backend == "nccl"  # torch's "nccl" backend is RCCL on ROCm
    assert args.dtype == "bf16x6"       # the parity-grade step is the headline
    args = b.make_parser().parse_args(["--gpus", "2", "--dist-backend", "gloo"])
    assert args.dist_backend == "gloo"
    assert b.init_distributed(args, 1, 0) is None  # N = 1: no process group


@pytest.mark.gpu
def test_bench_two_ranks_one_gpu(tmp_path):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env["MASTER_ADDR"] = "127.0.0.1"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--dist-backend", "gloo", "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out[-4000:]  # rank 0 only
    d = json.loads(lines[0])
    print(json.dumps({k: d[k] for k in ("value", "ms_per_step", "n_gpus", "elbo_per_img", "dtype")}))
    assert d["n_gpus"] == 2
    assert d["config"]["global_batch"] == 256 and d["config"]["per_gpu_batch"] == 128
    assert d["config"]["parallelism"] == "dp2"
    assert d["config"]["grad_allreduce"].startswith("per-step buckets")
    assert d["dtype"] == "bf16x6" and d["parity"] is True
    assert d["value"] > 0 and d["elbo_per_img"] == d["elbo_per_img"] and abs(d["elbo_per_img"]) < 1e6
