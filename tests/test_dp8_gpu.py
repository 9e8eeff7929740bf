"""BASELINE.json configs[3] on the HIP engine: CelebA 64x64, global batch 1024 sharded 8 x 128, one
averaged gradient per iteration (parallel.py).

Eight ranks share the one GPU of the test box (spawned before any GPU call; gloo over device
tensors -- RCCL refuses several ranks on one device, and the driver's 8-GPU bench covers RCCL over
xGMI).  Each rank runs the engine at B = 128 -- in the bench's headline mode bf16x6 (the fp32-grade split
step) and in bf16 -- on its contiguous shard of one 1024-image batch
through the bench's DP path: OverlappedAllReduce (per-step buckets exchanged from inside the
backward) + backward_apply (each bucket's clip + Adam right after its exchange).  Checked:
  * every rank's exchanged gradient equals the float64 mean of the 8 per-shard engine gradients to
    fp32 summation rounding (|d| <= 2e-6 * mean_r |g_r|, elementwise), and is bitwise the same on
    every rank;
  * the per-shard gradients are the single-process engine's: rank 0 re-runs the 8 shards one after
    another on a fresh engine, bitwise equal per shard;
  * the mean of the 8 shard losses equals the mean of the sequential run's losses, and each rank's
    DP-step loss equals its plain step's (the forward is deterministic);
  * all 8 replicas' parameters are bitwise equal after Adam, and equal to one Adam update of the
    sequential engine with the exchanged gradient."""
import json
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import pkg_mod

pytestmark = pytest.mark.gpu

WORLD, PER, LR, REG = 8, 128, 2e-4, 0.8


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _global_batch(cfg):
    g = torch.Generator().manual_seed(2024)
    x = torch.rand(WORLD * PER, cfg.height, cfg.width, cfg.channels, generator=g) * 2 - 1
    eps = torch.randn(cfg.mc_steps, WORLD * PER, cfg.latent_dim, generator=g)
    return x, eps


def _worker(rank, port, out_dir, dtype):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    cfgmod, SV, par = pkg_mod("config"), pkg_mod("sequential_vae").SequentialVAE, pkg_mod("parallel")
    cfg = cfgmod.preset("celeba", batch=PER, dtype=dtype)
    xg, eg = _global_batch(cfg)
    x = par.shard(xg, rank, WORLD).cuda().contiguous()
    eps = eg[:, rank * PER:(rank + 1) * PER].cuda().contiguous()
    net = SV(cfg, seed=0)
    n = net.n_live
    p_init = net.params.clone()
    # the plain per-shard step: this rank's gradient, the float64 mean over ranks and the sum of |g|
    net.forward(x, x, eps, REG)
    net.backward()
    torch.cuda.synchronize()
    loss_plain = net.loss_value()
    g_r = net.grads[:n].clone()
    mean64 = g_r.double()
    dist.all_reduce(mean64, op=dist.ReduceOp.SUM)
    mean64.mul_(1.0 / WORLD)
    abs64 = g_r.abs().double()
    dist.all_reduce(abs64, op=dist.ReduceOp.SUM)
    abs64.mul_(1.0 / WORLD)
    # the DP step of bench.py: overlapped per-bucket exchange + per-bucket Adam inside the backward
    net.enable_overlapped_allreduce(dist)
    net.forward(x, x, eps, REG)
    net.backward_apply(LR, 1)
    torch.cuda.synchronize()
    loss_dp = net.loss_value()
    ex = net.grads[:n].clone()
    err = (ex.double() - mean64).abs()
    ratio = float((err / (2e-6 * abs64 + 1e-30)).max())
    rel = float(err.norm() / mean64.norm())
    # bitwise equality across ranks: rank 0's exchanged gradient and parameters broadcast
    ex0, p0 = ex.clone(), net.params.clone()
    dist.broadcast(ex0, 0)
    dist.broadcast(p0, 0)
    same_ex, same_p = bool(torch.equal(ex0, ex)), bool(torch.equal(p0, net.params))
    losses = torch.tensor([loss_plain], dtype=torch.float64)
    allL = [torch.zeros(1, dtype=torch.float64) for _ in range(WORLD)]
    dist.all_gather(allL, losses)
    res = dict(rank=rank, loss_plain=loss_plain, loss_dp=loss_dp, ratio=ratio, rel=rel, same_ex=same_ex,
               same_p=same_p, finite=bool(torch.isfinite(ex).all() and torch.isfinite(net.params).all()),
               changed=float((net.params - p_init).abs().max()))
    if rank == 0:
        # one process, the 8 shards one after another on a fresh engine (same seed)
        ref = SV(cfg, seed=0)
        seq_sum = torch.zeros(n, dtype=torch.float64, device="cuda")
        seq_losses, shard_bitwise = [], True
        for r in range(WORLD):
            xr = par.shard(xg, r, WORLD).cuda().contiguous()
            er = eg[:, r * PER:(r + 1) * PER].cuda().contiguous()
            ref.forward(xr, xr, er, REG)
            ref.backward()
            torch.cuda.synchronize()
            seq_losses.append(ref.loss_value())
            seq_sum += ref.grads[:n].double()
            if r == 0:
                shard_bitwise = bool(torch.equal(ref.grads[:n], g_r))
        seq_mean = seq_sum / WORLD
        res["seq_vs_mean64"] = float(((seq_mean - mean64).norm() / mean64.norm()))
        res["shard0_bitwise"] = shard_bitwise
        res["seq_loss_mean"] = float(np.mean(seq_losses))
        res["dp_loss_mean"] = float(torch.cat(allL).mean())
        res["seq_losses_match"] = [float(a) for a in seq_losses] == [float(t) for t in torch.cat(allL)]
        # one Adam update of the sequential engine with the exchanged gradient = every replica
        ref.grads[:n].copy_(ex)
        ref.apply_gradients(LR, 1)
        torch.cuda.synchronize()
        res["adam_equal"] = bool(torch.equal(ref.params, net.params))
        ref.close()
    with open(os.path.join(out_dir, "r%d.json" % rank), "w") as f:
        json.dump(res, f)
    net.close()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("dtype", ["bf16x6", "bf16"])
def test_dp8_celeba_1024_sharded_on_engine(tmp_path, dtype):
    mp.spawn(_worker, args=(_free_port(), str(tmp_path), dtype), nprocs=WORLD, join=True)
    rs = [json.loads((tmp_path / ("r%d.json" % r)).read_text()) for r in range(WORLD)]
    r0 = rs[0]
    print("\nDP8 CelebA 1024 = 8 x 128 (%s engine, overlapped exchange + per-bucket Adam):" % dtype)
    for r in rs:
        print("  rank %d: loss %.6f (DP step %.6f); exchanged vs float64 mean: rel L2 %.2e, max |d| / (2e-6 mean|g|) "
              "%.3f; bitwise as rank 0: grad %s params %s" % (r["rank"], r["loss_plain"], r["loss_dp"], r["rel"],
                                                              r["ratio"], r["same_ex"], r["same_p"]))
    print("  sequential 8-shard run: gradient mean vs DP float64 mean rel %.2e, shard 0 bitwise %s, losses equal %s, "
          "mean loss %.6f vs %.6f; Adam with the exchanged gradient = replicas: %s" % (
              r0["seq_vs_mean64"], r0["shard0_bitwise"], r0["seq_losses_match"], r0["seq_loss_mean"],
              r0["dp_loss_mean"], r0["adam_equal"]))
    for r in rs:
        assert r["finite"] and r["changed"] > 0
        assert r["loss_dp"] == r["loss_plain"]
        assert r["ratio"] <= 1.0, r
        assert r["same_ex"] and r["same_p"]
    assert r0["shard0_bitwise"] and r0["seq_losses_match"]
    assert r0["seq_vs_mean64"] <= 1e-12
    assert abs(r0["seq_loss_mean"] - r0["dp_loss_mean"]) <= 1e-12 * abs(r0["seq_loss_mean"])
    assert r0["adam_equal"]
