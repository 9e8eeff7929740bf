"""Checkpoint / resume (SequentialVAE.save_checkpoint / load_checkpoint).

The reference saves and restores with tf.train.Saver (abstract_network.py:124-152): every
variable under its TF name plus the Adam slots "<name>/Adam" and "<name>/Adam_1".  The same
names go into a safetensors file here; a restored network must continue training exactly as the
one that was saved."""
import numpy as np
import pytest
import torch

from conftest import pkg_mod

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("preset,dtype", [("tiny", "bf16"), ("tiny_homog", "fp32")])
def test_save_load_resume(tmp_path, preset, dtype):
    cfgmod, SV = pkg_mod("config"), pkg_mod("sequential_vae").SequentialVAE
    cfg = cfgmod.preset(preset, batch=4, dtype=dtype)
    g = torch.Generator(device="cuda")
    g.manual_seed(21)
    x = torch.rand(cfg.batch, cfg.height, cfg.width, cfg.channels, device="cuda", generator=g) * 2 - 1
    a = SV(cfg, seed=3)
    for _ in range(2):
        a.train(x, x)
    path = str(tmp_path / "ckpt.safetensors")
    a.save_checkpoint(path)

    b = SV(cfg, seed=7)
    assert not torch.equal(a.params, b.params)
    b.load_checkpoint(path)
    assert b.iteration == a.iteration == 2
    assert b.learning_rate == a.learning_rate
    assert torch.equal(a.params, b.params)

    eps = torch.randn(cfg.mc_steps, cfg.batch, cfg.latent_dim, device="cuda", generator=g)
    for net in (a, b):
        net.iteration += 1
        net.forward(x, x, eps, 0.3)
        net.backward_apply(net.learning_rate, net.iteration)
    torch.cuda.synchronize()
    assert torch.equal(a.params, b.params)
    assert a.loss_value() == b.loss_value()

    from safetensors.numpy import load_file
    t = load_file(path)
    for p in a.table:
        assert t[p["name"]].shape == tuple(p["shape"])
        live = p["offset"] + p["size"] <= a.n_live
        assert (p["name"] + "/Adam" in t) == live and (p["name"] + "/Adam_1" in t) == live
    # TF's beta1_power after N updates is beta1^(N+1) (it starts at beta1)
    assert float(t["beta1_power"]) == pytest.approx(0.9 ** 3)
    assert float(t["beta2_power"]) == pytest.approx(0.999 ** 3)
    assert np.isfinite(t[a.table[0]["name"]]).all()
    a.close()
    b.close()


def test_checkpoint_without_metadata_recovers_adam_step(tmp_path):
    """A TF-converted checkpoint carries no metadata: the Adam step comes from beta1_power."""
    from safetensors.numpy import load_file, save_file
    cfg = pkg_mod("config").preset("tiny", batch=4)
    SV = pkg_mod("sequential_vae").SequentialVAE
    a = SV(cfg, seed=0)
    x = torch.rand(cfg.batch, cfg.height, cfg.width, cfg.channels, device="cuda") * 2 - 1
    for _ in range(3):
        a.train(x, x)
    path = str(tmp_path / "a.safetensors")
    a.save_checkpoint(path)
    bare = str(tmp_path / "bare.safetensors")
    save_file(load_file(path), bare)  # same tensors, no metadata
    b = SV(cfg, seed=5)
    b.load_checkpoint(bare)
    assert b.iteration == 3
    a.close()
    b.close()


def test_checkpoint_after_low_level_updates(tmp_path):
    """Adam steps taken through forward + backward_apply / apply_gradients (bench.py's and the DP
    loop's API, not train()) are counted too: beta1_power in the file matches the updates taken, and
    a resumed train() continues the bias correction from there."""
    from safetensors.numpy import load_file
    cfg = pkg_mod("config").preset("tiny", batch=4)
    SV = pkg_mod("sequential_vae").SequentialVAE
    a = SV(cfg, seed=0)
    x = torch.rand(cfg.batch, cfg.height, cfg.width, cfg.channels, device="cuda") * 2 - 1
    a.forward(x, x, None, 1.0)
    a.backward_apply()           # Adam step 1
    a.forward(x, x, None, 1.0)
    a.backward()
    a.apply_gradients()          # Adam step 2
    assert a.adam_updates == 2
    path = str(tmp_path / "low.safetensors")
    a.save_checkpoint(path)
    t = load_file(path)
    assert float(t["beta1_power"]) == pytest.approx(0.9 ** 3)
    assert float(t["beta2_power"]) == pytest.approx(0.999 ** 3)
    b = SV(cfg, seed=5)
    b.load_checkpoint(path)
    assert b.adam_updates == 2
    eps = torch.randn(cfg.mc_steps, cfg.batch, cfg.latent_dim, device="cuda")
    a.train(x, x, eps=eps)
    b.train(x, x, eps=eps)
    assert a.adam_updates == b.adam_updates == 3
    torch.cuda.synchronize()
    assert torch.equal(a.params, b.params)
    a.close()
    b.close()
