"""Step time of the CelebA B=128 engine with and without an RCCL process group in the process (and with the
overlapped per-bucket exchange hook on one rank): does the communicator's presence slow the engine?

    python tools/dist_overhead.py [none|pg|pg_hook] [steps]
Run one mode per process (GPU_MAX_HW_QUEUES etc. from the environment)."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import importlib  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "none"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
PKG = "sequential-variational-autoencoder_amd"
torch.cuda.set_device(0)
dist = None
if mode != "none":
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
cfg = importlib.import_module(PKG + ".config").preset("celeba", batch=128, dtype="bf16x6")
net = importlib.import_module(PKG + ".sequential_vae").SequentialVAE(cfg, seed=0)
if mode == "pg_hook":
    net.enable_overlapped_allreduce(dist, force=True)
x = torch.rand(128, 64, 64, 3, device="cuda") * 2 - 1
it = 0
def run(n):
    global it
    for _ in range(n):
        it += 1
        net.forward(x, x, None, 0.5)
        net.backward_apply(2e-4, it)
    torch.cuda.synchronize()
run(40)
best = 1e9
for _ in range(3):
    t0 = time.perf_counter()
    run(steps)
    best = min(best, (time.perf_counter() - t0) / steps * 1e3)
print("%s HWQ=%s: %.3f ms/step" % (mode, os.environ.get("GPU_MAX_HW_QUEUES", "default"), best), flush=True)
net.close()
if dist is not None:
    dist.destroy_process_group()
