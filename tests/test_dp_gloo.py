"""Data-parallel path on CPU (gloo, world_size 2, 4 and 8): per-shard BN semantics + one
all-reduce of the flat gradient (SURVEY.md §8e parity rule):
  N-rank loss  = mean over shards of the single-process loss of each shard
  N-rank grad  = mean over shards of the per-shard gradients
The per-shard compute is the CPU twin (the GPU engine is covered by test_engine_gpu);
the exchange is the product's parallel.allreduce_hook."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import pkg_mod
from oracle import spec, torch_twin


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _shard_grads(rank, world, gx, gt, eps_all):
    cd = spec.make_config("tiny", batch=gx.shape[0] // world)
    table, struct, params = spec.init_params(cd, seed=0)
    par = pkg_mod("parallel")
    x = par.shard(torch.from_numpy(gx), rank, world).numpy()
    t = par.shard(torch.from_numpy(gt), rank, world).numpy()
    eps = eps_all[:, rank * cd["batch"]:(rank + 1) * cd["batch"]]
    tw = torch_twin.Twin(cd, struct, params, dtype=torch.float64)
    o = tw.step(x, t, eps, 0.5)
    names = [p["name"] for p in table]
    flat = torch.from_numpy(np.concatenate([o["grads"][n].ravel() for n in names]))
    return o["loss"], flat


def _worker(rank, world, port, gx, gt, eps_all, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    par = pkg_mod("parallel")
    loss, flat = _shard_grads(rank, world, gx, gt, eps_all)
    hook = par.allreduce_hook(dist)
    hook(flat)
    mloss = par.mean_scalar(dist, loss, torch.device("cpu"))
    np.save(os.path.join(out_dir, "g%d.npy" % rank), flat.numpy())
    np.save(os.path.join(out_dir, "l%d.npy" % rank), np.array([mloss, loss]))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_dp_allreduce_matches_shard_mean(tmp_path, world):
    B = 4 * world
    cd = spec.make_config("tiny", batch=B)
    gx, gt, eps_all = spec.make_inputs(cd, batch=B)
    mp.spawn(_worker, args=(world, _free_port(), gx, gt, eps_all, str(tmp_path)), nprocs=world, join=True)
    ref = [_shard_grads(r, world, gx, gt, eps_all) for r in range(world)]
    mean_g = sum(f for _, f in ref) / world
    mean_l = sum(l for l, _ in ref) / world
    for r in range(world):
        g = np.load(tmp_path / ("g%d.npy" % r))
        ml, own = np.load(tmp_path / ("l%d.npy" % r))
        np.testing.assert_allclose(g, mean_g.numpy(), rtol=1e-12, atol=1e-15)
        assert abs(ml - mean_l) <= 1e-12 * abs(mean_l)
        assert abs(own - ref[r][0]) <= 1e-12 * abs(own)
    # replicas identical after the exchange
    np.testing.assert_array_equal(np.load(tmp_path / "g0.npy"), np.load(tmp_path / "g1.npy"))


def test_shard_is_contiguous():
    par = pkg_mod("parallel")
    b = torch.arange(1024)
    parts = [par.shard(b, r, 8) for r in range(8)]
    assert all(len(p) == 128 for p in parts)
    assert torch.equal(torch.cat(parts), b)


@pytest.mark.parametrize("preset", ["tiny", "celeba", "lsun"])
def test_step_buckets_tile_the_live_gradient(preset):
    """The overlapped all-reduce's buckets: theta_t in backward order T-1..0, then phi; together
    they cover [0, n_live) exactly once."""
    par, w, cfgmod = pkg_mod("parallel"), pkg_mod("weights"), pkg_mod("config")
    cfg = cfgmod.preset(preset)
    table, _, n_live = w.param_table(cfg)
    steps, phi = par.step_buckets(table, n_live)
    assert [t for t, _, _ in steps] == list(range(cfg.mc_steps - 1, -1, -1))
    spans = sorted([(lo, hi) for _, lo, hi in steps] + [phi])
    assert spans[0][0] == 0 and spans[-1][1] == n_live
    assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))


class _FakeNet:  # the hook's view of SequentialVAE without the GPU engine
    def __init__(self, grads, table, n_live):
        self.grads, self.table, self.n_live, self.ctx = grads, table, n_live, None


def _overlap_worker(rank, world, port, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    par, w, cfgmod = pkg_mod("parallel"), pkg_mod("weights"), pkg_mod("config")
    cfg = cfgmod.preset("tiny")
    table, n_total, n_live = w.param_table(cfg)
    g = torch.from_numpy(np.random.default_rng(rank).standard_normal(n_total).astype(np.float32))
    net = _FakeNet(g, table, n_live)
    ov = par.OverlappedAllReduce(net, dist)
    for t in range(cfg.mc_steps - 1, -1, -1):  # the engine's call order
        ov._on_step(None, t)
    ov._on_step(None, -1)
    ov.check()
    np.save(os.path.join(out_dir, "o%d.npy" % rank), g.numpy())
    dist.destroy_process_group()


def test_overlapped_allreduce_equals_mean(tmp_path):
    world = 2
    mp.spawn(_overlap_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    w, cfgmod = pkg_mod("weights"), pkg_mod("config")
    _, n_total, n_live = w.param_table(cfgmod.preset("tiny"))
    src = [np.random.default_rng(r).standard_normal(n_total).astype(np.float32) for r in range(world)]
    mean = (src[0][:n_live] + src[1][:n_live]) * np.float32(0.5)
    for r in range(world):
        o = np.load(tmp_path / ("o%d.npy" % r))
        np.testing.assert_allclose(o[:n_live], mean, rtol=1e-6, atol=1e-7)
        np.testing.assert_array_equal(o[n_live:], src[r][n_live:])  # dead tail untouched
    np.testing.assert_array_equal(np.load(tmp_path / "o0.npy")[:n_live], np.load(tmp_path / "o1.npy")[:n_live])


def _twin_flat(rank, world, gx, gt, eps_all, table, n_total):
    """Rank `rank`'s shard of the global batch through the fp64 twin; its gradient laid out in the
    engine's flat buffer (weights.param_table offsets), so the product's buckets apply to it."""
    cd = spec.make_config("tiny", batch=gx.shape[0] // world)
    _, struct, params = spec.init_params(cd, seed=0)
    par = pkg_mod("parallel")
    x = par.shard(torch.from_numpy(gx), rank, world).numpy()
    t = par.shard(torch.from_numpy(gt), rank, world).numpy()
    eps = eps_all[:, rank * cd["batch"]:(rank + 1) * cd["batch"]]
    o = torch_twin.Twin(cd, struct, params, dtype=torch.float64).step(x, t, eps, 0.5)
    flat = torch.zeros(n_total, dtype=torch.float64)
    for p in table:
        flat[p["offset"]:p["offset"] + p["size"]] = torch.from_numpy(np.ravel(o["grads"][p["name"]]))
    return o["loss"], flat


def _overlap_twin_worker(rank, world, port, gx, gt, eps_all, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    par, w, cfgmod = pkg_mod("parallel"), pkg_mod("weights"), pkg_mod("config")
    table, n_total, n_live = w.param_table(cfgmod.preset("tiny"))
    loss, flat = _twin_flat(rank, world, gx, gt, eps_all, table, n_total)
    ov = par.OverlappedAllReduce(_FakeNet(flat, table, n_live), dist)
    T = cfgmod.preset("tiny").mc_steps
    for t in range(T - 1, -1, -1):  # the engine's call order: theta_t buckets, then phi
        ov._on_step(None, t)
    ov._on_step(None, -1)
    ov.check()
    np.save(os.path.join(out_dir, "tg%d.npy" % rank), flat.numpy())
    np.save(os.path.join(out_dir, "tl%d.npy" % rank), np.array([par.mean_scalar(dist, loss, torch.device("cpu")), loss]))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 8])
def test_overlapped_buckets_on_twin_gradients(tmp_path, world):
    """The DP8 configuration's exchange on real gradients: a global batch of 128*world images
    (1024 -> 8 x 128 at world 8) in contiguous shards, each rank's fp64 twin gradient in the flat
    engine layout, the per-step buckets of parallel.OverlappedAllReduce in the engine's call order.
    Every replica ends with the mean of the per-shard gradients (the dead tail untouched) and the
    mean of the per-shard losses (SURVEY §8e parity rule)."""
    B = 128 * world
    cd = spec.make_config("tiny", batch=B)
    gx, gt, eps_all = spec.make_inputs(cd, batch=B)
    mp.spawn(_overlap_twin_worker, args=(world, _free_port(), gx, gt, eps_all, str(tmp_path)), nprocs=world, join=True)
    w, cfgmod = pkg_mod("weights"), pkg_mod("config")
    table, n_total, n_live = w.param_table(cfgmod.preset("tiny"))
    torch.set_num_threads(max(1, min(8, torch.get_num_threads())))
    ref = [_twin_flat(r, world, gx, gt, eps_all, table, n_total) for r in range(world)]
    mean_g = (sum(f for _, f in ref) / world).numpy()
    mean_l = sum(l for l, _ in ref) / world
    g0 = np.load(tmp_path / "tg0.npy")
    for r in range(world):
        g = np.load(tmp_path / ("tg%d.npy" % r))
        np.testing.assert_allclose(g[:n_live], mean_g[:n_live], rtol=1e-12, atol=1e-15)
        # the dead / zero-gradient tail is not exchanged: each rank keeps its own (round-off) values
        np.testing.assert_allclose(g[n_live:], ref[r][1].numpy()[n_live:], rtol=0, atol=1e-12)
        np.testing.assert_array_equal(g[:n_live], g0[:n_live])  # replicas bitwise equal
        ml, own = np.load(tmp_path / ("tl%d.npy" % r))
        assert abs(ml - mean_l) <= 1e-12 * abs(mean_l)
        assert abs(own - ref[r][0]) <= 1e-12 * abs(own)
