"""Data parallelism over the batch.

One process per GPU; each rank owns a full parameter replica and a contiguous
B-image shard.  BatchNorm statistics are per shard (exactly the reference
computation at B images per shard; SyncBN is a non-goal).  The only exchange is
ONE all-reduce(AVG) of the live region of the flat fp32 gradient buffer
(RCCL over xGMI for backend "nccl"; gloo for the CPU tests), after which every
rank applies the identical clip+Adam update, so replicas stay bitwise equal.

The reference has no collective at all; this is the added DP path.
"""
import re
from contextlib import nullcontext as _nullctx

import torch

from . import _lib


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


_STEP = re.compile(r"^theta/generative(?:_encoder)?_step_(\d+)/")


def step_buckets(table, n_live):
    """Gradient buckets of the flat buffer in the order the backward completes them.

    The inhomogeneous chain gives every step its own generator/encoder weights
    (sequential_vae.py:1683-1687,1757-1761 with share_theta off), laid out contiguously per step
    after all recognition weights ("phi/inference_step_t", batched backward, finishes last).
    Returns ([(t, lo, hi) for t = T-1..0], (lo, hi) of phi); the ranges tile [0, n_live)."""
    # the live region [0, n_live): dead tensors and the exactly-zero gradients of BN-followed
    # biases (FLAG_ZERO_GRAD) sit after it and are not exchanged
    live = [p for p in table if not p["dead"] and p["offset"] < n_live]
    keys = []
    for p in live:
        m = _STEP.match(p["name"])
        keys.append(("theta", int(m.group(1))) if m else ("phi", -1))
    starts = {}
    for k, p in zip(keys, live):
        starts[k] = min(starts.get(k, p["offset"]), p["offset"])
    order = sorted(starts.items(), key=lambda kv: kv[1])
    ranges = {}
    for i, (k, lo) in enumerate(order):
        hi = order[i + 1][1] if i + 1 < len(order) else n_live
        ranges[k] = (lo, hi)
    for k, p in zip(keys, live):  # every tensor inside its own bucket
        lo, hi = ranges[k]
        assert lo <= p["offset"] and p["offset"] + p["size"] <= hi, (p["name"], k)
    if ("phi", -1) not in ranges or ranges[("phi", -1)][0] != 0:
        raise ValueError("unexpected layout: recognition weights must come first")
    steps = sorted((t for (kind, t) in ranges if kind == "theta"), reverse=True)
    return [(t,) + ranges[("theta", t)] for t in steps], ranges[("phi", -1)]


class OverlappedAllReduce:
    """Bucketed gradient all-reduce overlapped with the backward (svae_set_backward_hook).

    After the backward of chain step t the engine calls back; step t's generator/encoder
    gradients are then complete and one all_reduce of that bucket is enqueued on the engine's
    hook stream (ordered after the step's kernels on both engine streams), so RCCL moves it over
    xGMI while steps t-1..0 still compute.  The recognition bucket follows the batched
    recognition backward on the caller's stream; the caller's stream then waits for every
    bucket.  Same result as one all-reduce of the whole buffer (elementwise sums)."""

    def __init__(self, net, dist, group=None, force=False):
        self.dist, self.group = dist, group
        self.world = dist.get_world_size(group)
        self.grads = net.grads
        self.n_live = net.n_live
        self.buckets, self.phi = step_buckets(net.table, net.n_live)
        self.avg = dist.get_backend(group) == "nccl"  # ReduceOp.AVG (RCCL); gloo: SUM then scale
        self.pending = []
        self.error = None
        self.eager = False  # svae_backward_adam: each bucket's update follows its exchange on the hook stream
        self.done = []
        self.side = None
        self.by_t = {t: (lo, hi) for t, lo, hi in self.buckets}
        self._cb = _lib.STEP_HOOK(self._on_step)  # keep the ctypes thunk alive
        if getattr(net, "ctx", None) is not None and (self.world > 1 or force):
            _lib.check(net.L.svae_set_backward_hook(net.ctx, self._cb, None), net.ctx)
            self.side = torch.cuda.ExternalStream(net.L.svae_hook_stream(net.ctx), device=net.device)

    def _reduce(self, lo, hi):
        op = self.dist.ReduceOp.AVG if self.avg else self.dist.ReduceOp.SUM
        self.pending.append(self.dist.all_reduce(self.grads[lo:hi], op=op, group=self.group, async_op=True))

    def _on_step(self, _user, t):
        try:
            if t >= 0:
                lo, hi = self.by_t[t]
                with torch.cuda.stream(self.side) if self.side is not None else _nullctx():
                    self._reduce(lo, hi)
                    if self.eager:  # the engine enqueues this bucket's Adam on the hook stream next
                        self.pending.pop().wait()
                        if not self.avg:
                            self.grads[lo:hi].mul_(1.0 / self.world)
                        self.done.append((lo, hi))
            else:
                self._reduce(*self.phi)
                for w in self.pending:
                    w.wait()
                self.pending = []
                if not self.avg:
                    if self.done:
                        for lo, hi in [self.phi] + [(lo, hi) for _, lo, hi in self.buckets if (lo, hi) not in self.done]:
                            self.grads[lo:hi].mul_(1.0 / self.world)
                    else:
                        self.grads[:self.n_live].mul_(1.0 / self.world)
                self.done = []
        except BaseException as e:  # a ctypes callback cannot raise into C: re-raised by check()
            self.error = e

    def check(self):
        if self.error is not None:
            e, self.error = self.error, None
            raise e


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
