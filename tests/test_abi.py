"""CPU checks of the drop-in boundary: the C-ABI library builds for gfx950, loads,
exports every entry point include/svae_hip.h declares, and its (pure-host)
parameter layout equals the oracle's restatement of the reference variable table."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import ROOT, pkg_mod
from oracle import spec, weightgen


def _header_symbols(name="svae_hip.h"):
    txt = open(os.path.join(ROOT, "include", name)).read()
    return sorted(set(re.findall(r"\b(svae_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_header_symbols(built_lib):
    lib = ctypes.CDLL(built_lib)
    syms = _header_symbols()
    assert len(syms) >= 15
    for s in syms:
        assert hasattr(lib, s), s
    assert sorted(pkg_mod("_lib").EXPORTED) == syms


def test_library_embeds_its_source_hash(built_lib):
    """the library carries the hash of the sources it was compiled from (build.py
    src_hash over csrc/* and include/*), as svae_build_hash() and as the literal build() reads from the
    file; _lib refuses a library whose hash is not the tree's, so no stale binary is ever tested."""
    build = pkg_mod("build")
    want = build.src_hash()
    assert re.fullmatch(r"[0-9a-f]{16}", want)
    assert build.embedded_hash(built_lib) == want
    lib = ctypes.CDLL(built_lib)
    lib.svae_build_hash.restype = ctypes.c_char_p
    assert lib.svae_build_hash().decode() == want
    knobs = build.build(knobs=True)
    assert build.embedded_hash(knobs) == want


def test_loader_refuses_a_library_from_other_sources(built_lib, tmp_path, monkeypatch):
    """A copy of the library whose embedded hash differs from the tree's does not load through _lib."""
    L = pkg_mod("_lib")
    data = open(built_lib, "rb").read()
    i = data.find(b"SVAE_SRC_HASH=")
    assert i >= 0
    old = data[i + 14:i + 30]
    bad = bytes(ord("0") if c != ord("0") else ord("1") for c in old)
    stale = tmp_path / "libsvae_hip.so"
    stale.write_bytes(data[:i + 14] + bad + data[i + 30:])
    monkeypatch.delenv("SVAE_LIB", raising=False)
    with pytest.raises(RuntimeError, match="built from other sources"):
        L._load(str(stale))


def test_library_exports_pcnn_symbols(built_lib):
    """include/svae_pcnn.h (the PixelCNN++ head): every entry point is exported and
    has a ctypes signature."""
    lib = ctypes.CDLL(built_lib)
    syms = _header_symbols("svae_pcnn.h")
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(lib, s), s
    assert sorted(pkg_mod("_lib").PCNN_EXPORTED) == syms


@pytest.mark.parametrize("preset", ["tiny", "celeba", "lsun", "mnist_1step"])
def test_layout_matches_oracle_table(built_lib, preset):
    W = pkg_mod("weights")
    cfg = pkg_mod("config").preset(preset)
    table, n_total, n_live = W.param_table(cfg)
    otab, _ = spec.build_params(spec.make_config(preset))
    key = lambda p: (p["name"], tuple(p["shape"]), p["dead"], p["zero_grad"], p["init"])
    assert sorted(map(key, table)) == sorted(map(key, otab))
    # 64-float aligned, non-overlapping spans inside [0, n_total); live tensors first
    spans = sorted((p["offset"], p["offset"] + p["size"], p["dead"] or p["zero_grad"]) for p in table)
    pos = 0
    for a, b, frozen in spans:
        assert a % 64 == 0 and a >= pos
        assert (a >= n_live) == frozen
        pos = b
    assert pos <= n_total and n_total - pos < 64 and n_live % 64 == 0
    # recognition blocks: identical per-step layout at a constant stride (batched launches)
    off = {p["name"]: p["offset"] for p in table}
    t0 = [n for n in off if n.startswith("phi/inference_step_0/") and n in off and off[n] < n_live]
    if cfg.mc_steps > 1:
        stride = off[t0[0].replace("step_0", "step_1")] - off[t0[0]]
        for n in t0:
            assert off[n.replace("step_0", "step_1")] - off[n] == stride


def test_weight_generators_agree(built_lib):
    W = pkg_mod("weights")
    cfg = pkg_mod("config").preset("tiny")
    table, _, _ = W.param_table(cfg)
    for p in table:
        a = W.init_value(p["name"], p["shape"], p["init"], 7)
        b = weightgen.generate(p["name"], p["shape"], p["init"], 7).ravel()
        np.testing.assert_array_equal(a, b)


def test_bad_config_rejected(built_lib):
    L = pkg_mod("_lib")
    cfg = pkg_mod("config").preset("tiny", batch=1).to_c()
    n = ctypes.c_int64()
    rc = L.lib().svae_param_count(ctypes.byref(cfg), ctypes.byref(n), None, None)
    assert rc == -1
    assert b"batch" in L.lib().svae_last_error(None)


def test_homog_layout_matches_oracle_sharing(built_lib):
    """Public parameter table of the homogeneous presets = the oracle's restatement of TF's
    variable sharing (names and shapes); the live region precedes the frozen tail."""
    from oracle import spec
    w, cfgmod = pkg_mod("weights"), pkg_mod("config")
    for theta, phi in [(True, True), (True, False), (False, True)]:
        cfg = cfgmod.preset("tiny", share_theta_weights=theta, share_phi_weights=phi)
        table, n_total, n_live = w.param_table(cfg)
        ref = {p["name"]: tuple(p["shape"]) for p in spec.shared_table(spec.make_config("tiny"), theta, phi)}
        assert {p["name"]: tuple(p["shape"]) for p in table} == ref
        for p in table:
            assert (p["offset"] < n_live) == (not p["zero_grad"]), p["name"]
            assert p["offset"] + p["size"] <= n_total


@pytest.mark.parametrize("preset", ["tiny", "celeba"])
def test_stddev_network_layout_matches_oracle(built_lib, preset):
    """predict_generator_noise adds stddevs_prediction's variables to every generator scope
    (sequential_vae.py:1866-1875): the engine's table equals the oracle's, names and TF order."""
    W, cfgmod = pkg_mod("weights"), pkg_mod("config")
    cfg = cfgmod.preset(preset, add_noise_to_chain=True, predict_generator_noise=True)
    table, n_total, n_live = W.param_table(cfg)
    otab, _ = spec.build_params(spec.make_config(preset, add_noise_to_chain=True, predict_generator_noise=True))
    key = lambda p: (p["name"], tuple(p["shape"]), p["dead"], p["zero_grad"], p["init"])
    assert sorted(map(key, table)) == sorted(map(key, otab))
    names = [p["name"] for p in table]
    assert "theta/generative_step_0/Conv_5/weights" in names and "theta/generative_step_0/Conv_5/biases" in names
    # homogeneous chain: the stddev network is shared like the rest of the generator (:1683-1687)
    cfg = cfgmod.preset(preset, add_noise_to_chain=True, predict_generator_noise=True, share_theta_weights=True,
                        share_phi_weights=True)
    table, _, _ = W.param_table(cfg)
    cd = spec.make_config(preset, add_noise_to_chain=True, predict_generator_noise=True)
    ref = {p["name"]: tuple(p["shape"]) for p in spec.shared_table(cd, True, True)}
    assert {p["name"]: tuple(p["shape"]) for p in table} == ref


def test_chain_variant_configs_rejected(built_lib):
    L = pkg_mod("_lib")
    cfgmod = pkg_mod("config")
    for over, msg in [(dict(predict_generator_noise=True), b"add_noise_to_chain"),
                      (dict(add_noise_to_chain=True, predict_generator_noise=True,
                            predict_generator_stddev_filter_sizes=(5, 9)), b"stddev_filter_sizes")]:
        c = cfgmod.preset("tiny", **over).to_c()
        n = ctypes.c_int64()
        assert L.lib().svae_param_count(ctypes.byref(c), ctypes.byref(n), None, None) == -1
        assert msg in L.lib().svae_last_error(None)
    # noise_stddevs follow the reference list (sequential_vae.py:239), indexed by step
    c = cfgmod.preset("tiny", add_noise_to_chain=True).to_c()
    assert [c.noise_stddevs[t] for t in range(4)] == [0.5, 0.25, 0.125, 0.0]
