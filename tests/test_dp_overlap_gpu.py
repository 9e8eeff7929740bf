"""Overlapped data-parallel gradient exchange on the GPU engine (parallel.OverlappedAllReduce).

Two ranks share the one GPU of the test box (gloo backend over CUDA tensors: RCCL refuses two
ranks on one device); each runs the HIP training step on its own shard.  The per-step buckets
all-reduced from inside svae_backward (engine hook, side-stream ordering) must give exactly
the mean of the per-rank gradients that a plain backward produces (one exchange afterwards)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import pkg_mod

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, preset, dtype, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfgmod, SV = pkg_mod("config"), pkg_mod("sequential_vae").SequentialVAE
    cfg = cfgmod.preset(preset, batch=4, dtype=dtype)
    net = SV(cfg, seed=0)
    g = torch.Generator(device="cuda")
    g.manual_seed(100 + rank)
    x = torch.rand(cfg.batch, cfg.height, cfg.width, cfg.channels, device="cuda", generator=g) * 2 - 1
    eps = torch.randn(cfg.mc_steps, cfg.batch, cfg.latent_dim, device="cuda", generator=g)
    net.forward(x, x, eps, 0.7)
    net.backward()
    ref = net.grads[:net.n_live].clone()
    dist.all_reduce(ref, op=dist.ReduceOp.SUM)
    ref.mul_(1.0 / world)
    net.enable_overlapped_allreduce(dist)
    net.forward(x, x, eps, 0.7)
    net.backward()
    torch.cuda.synchronize()
    np.save(os.path.join(out_dir, "ref%d.npy" % rank), ref.cpu().numpy())
    np.save(os.path.join(out_dir, "ov%d.npy" % rank), net.grads[:net.n_live].cpu().numpy())
    net.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("preset,dtype", [("tiny", "fp32"), ("celeba", "bf16")])
def test_overlapped_allreduce_matches_single_exchange(tmp_path, preset, dtype):
    world = 2
    mp.get_context("spawn")
    mp.spawn(_worker, args=(world, _free_port(), preset, dtype, str(tmp_path)), nprocs=world, join=True)
    for r in range(world):
        ref, ov = np.load(tmp_path / ("ref%d.npy" % r)), np.load(tmp_path / ("ov%d.npy" % r))
        assert np.isfinite(ov).all()
        np.testing.assert_array_equal(ov, ref)
    np.testing.assert_array_equal(np.load(tmp_path / "ov0.npy"), np.load(tmp_path / "ov1.npy"))


def _fused_worker(rank, world, port, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfgmod, SV = pkg_mod("config"), pkg_mod("sequential_vae").SequentialVAE
    cfg = cfgmod.preset("tiny", batch=4, dtype="bf16")
    ref, net = SV(cfg, seed=0), SV(cfg, seed=0)
    g = torch.Generator(device="cuda")
    g.manual_seed(200 + rank)
    x = torch.rand(cfg.batch, cfg.height, cfg.width, cfg.channels, device="cuda", generator=g) * 2 - 1
    eps = torch.randn(cfg.mc_steps, cfg.batch, cfg.latent_dim, device="cuda", generator=g)
    for it in (1, 2):  # one exchange after the backward, then Adam
        ref.forward(x, x, eps, 0.7)
        ref.backward()
        gr = ref.grads[:ref.n_live]
        dist.all_reduce(gr, op=dist.ReduceOp.SUM)
        gr.mul_(1.0 / world)
        ref.apply_gradients(1e-3, it)
    net.enable_overlapped_allreduce(dist)
    for it in (1, 2):  # per-bucket exchange + Adam inside the backward
        net.forward(x, x, eps, 0.7)
        net.backward_apply(1e-3, it)
    torch.cuda.synchronize()
    np.save(os.path.join(out_dir, "fref%d.npy" % rank), ref.params.cpu().numpy())
    np.save(os.path.join(out_dir, "fov%d.npy" % rank), net.params.cpu().numpy())
    ref.close()
    net.close()
    dist.destroy_process_group()


def test_overlapped_allreduce_with_fused_adam(tmp_path):
    """backward_apply under the overlapped exchange: every bucket's Adam runs after that bucket's
    all-reduce on the hook stream; parameters equal exchange-then-Adam bit for bit on both ranks."""
    world = 2
    mp.spawn(_fused_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    for r in range(world):
        np.testing.assert_array_equal(np.load(tmp_path / ("fov%d.npy" % r)), np.load(tmp_path / ("fref%d.npy" % r)))
    np.testing.assert_array_equal(np.load(tmp_path / "fov0.npy"), np.load(tmp_path / "fov1.npy"))


def _nccl_worker(rank, port, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    cfgmod, SV = pkg_mod("config"), pkg_mod("sequential_vae").SequentialVAE
    cfg = cfgmod.preset("tiny", batch=4)
    net = SV(cfg, seed=0)
    x = torch.rand(cfg.batch, cfg.height, cfg.width, cfg.channels, device="cuda") * 2 - 1
    eps = torch.randn(cfg.mc_steps, cfg.batch, cfg.latent_dim, device="cuda")
    net.forward(x, x, eps, 1.0)
    net.backward()
    ref = net.grads.clone()
    ov = net.enable_overlapped_allreduce(dist, force=True)  # RCCL path, ReduceOp.AVG, hook stream
    assert ov.avg and ov.side is not None
    for _ in range(2):
        net.forward(x, x, eps, 1.0)
        net.backward()
    torch.cuda.synchronize()
    np.save(os.path.join(out_dir, "d.npy"), (net.grads - ref).abs().max().cpu().numpy())
    net.close()
    dist.destroy_process_group()


def test_overlapped_allreduce_rccl_single_rank(tmp_path):
    """The RCCL (nccl backend) form of the hook: AVG over one rank leaves the gradient bitwise
    unchanged; exercises the collective on the engine's hook stream from inside svae_backward."""
    mp.spawn(_nccl_worker, args=(_free_port(), str(tmp_path)), nprocs=1, join=True)
    assert float(np.load(tmp_path / "d.npy")) == 0.0
