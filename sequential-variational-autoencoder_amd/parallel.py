"""Data parallelism over the batch.

One process per GPU; each rank owns a full parameter replica and a contiguous
B-image shard.  BatchNorm statistics are per shard (exactly the reference
computation at B images per shard; SyncBN is a non-goal).  The only exchange is
ONE all-reduce(AVG) of the live region of the flat fp32 gradient buffer
(RCCL over xGMI for backend "nccl"; gloo for the CPU tests), after which every
rank applies the identical clip+Adam update, so replicas stay bitwise equal.

The reference has no collective at all; this is the added DP path.
"""
import torch


def allreduce_hook(dist, group=None, bucket_elems=None):
    """Gradient hook for SequentialVAE(grad_hook=...): averages the live gradient
    region across ranks.  ``bucket_elems`` splits the buffer into several
    all-reduces (same result) to let RCCL pipeline them; None = one call."""
    def hook(flat_grads: torch.Tensor):
        world = dist.get_world_size(group)
        if world == 1:
            return
        if bucket_elems:
            for chunk in torch.split(flat_grads, bucket_elems):
                dist.all_reduce(chunk, op=dist.ReduceOp.SUM, group=group)
        else:
            dist.all_reduce(flat_grads, op=dist.ReduceOp.SUM, group=group)
        flat_grads.mul_(1.0 / world)
    return hook


def shard(batch: torch.Tensor, rank: int, world: int) -> torch.Tensor:
    """Contiguous batch shard of a global batch (1024 -> 8 x 128)."""
    n = batch.shape[0]
    assert n % world == 0, "global batch must divide evenly"
    per = n // world
    return batch[rank * per:(rank + 1) * per]


def mean_scalar(dist, value: float, device, group=None) -> float:
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return float(t.item()) / dist.get_world_size(group)
