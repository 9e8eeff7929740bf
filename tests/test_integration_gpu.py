"""The bare ctypes binding printed in INTEGRATION.md §2 is real code: it is extracted from
the document, run in a torch-free subprocess against the in-tree libsvae_hip.so, and must
reproduce the torch-based mirror (SequentialVAE) bit for bit: same initial parameters,
same on-device Philox eps sequence, deterministic kernels."""
import os
import re
import subprocess
import sys
import textwrap

import numpy as np
import pytest
import torch

from conftest import PKG_NAME, ROOT, pkg_mod

pytestmark = pytest.mark.gpu

DRIVER = r'''
import sys, numpy as np, ctypes
{stub}
cfg = svae_config()
cfg.batch, cfg.height, cfg.width, cfg.channels, cfg.levels, cfg.mc_steps = 4, 32, 32, 3, 4, 3
for i, f in enumerate([3, 8, 8, 16, 24, 16]): cfg.filter_sizes[i] = f
for i, d in enumerate([2, 2, 3, 2]): cfg.latent_dims[i] = d
cfg.intermediate_reconstruction, cfg.first_step_loss_coeff, cfg.latent_prior_stddev = 1, 1.0, 1.0
cfg.latent_mean_clip, cfg.range_lo, cfg.range_hi = float("inf"), -1.0, 1.0
cfg.min_highway, cfg.max_highway, cfg.dtype = 0.0, 1.0, 0
P0 = np.load(sys.argv[1]); x = np.load(sys.argv[2])
net = HipSequentialVAE(cfg, P0)
losses = [net.train(x, x) for _ in range(3)]
np.save(sys.argv[3], np.array(losses, np.float64)); np.save(sys.argv[4], net.test(x))
'''


def _stub():
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    code = re.search(r"```python\n(.*?)```", doc, re.S).group(1)
    lib = os.path.join(ROOT, PKG_NAME, "libsvae_hip.so")
    code = code.replace('ctypes.CDLL("libsvae_hip.so")', "ctypes.CDLL(%r)" % lib)
    return code.replace('ctypes.CDLL("libamdhip64.so")', 'ctypes.CDLL("/opt/rocm/lib/libamdhip64.so")')


def test_integration_stub_matches_mirror(tmp_path):
    cfg = pkg_mod("config").preset("tiny", batch=4)
    P0 = pkg_mod("weights").init_flat(cfg, 0)
    x = np.random.default_rng(5).uniform(-1, 1, (4, 32, 32, 3)).astype(np.float32)
    f = {k: str(tmp_path / (k + ".npy")) for k in ("p", "x", "loss", "out")}
    np.save(f["p"], P0)
    np.save(f["x"], x)
    script = tmp_path / "drive.py"
    script.write_text(DRIVER.format(stub=_stub()))
    env = dict(os.environ)
    r = subprocess.run([sys.executable, str(script), f["p"], f["x"], f["loss"], f["out"]], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    net = pkg_mod("sequential_vae").SequentialVAE(cfg, seed=0)
    assert np.array_equal(net.params.cpu().numpy(), P0)
    losses = [net.train(x, x) for _ in range(3)]
    out = net.test(x)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(np.load(f["loss"]), np.array(losses))
    np.testing.assert_array_equal(np.load(f["out"]), out)
