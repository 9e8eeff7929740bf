"""MI355X-native Sequential-VAE training-step engine (HIP / CDNA4, gfx950).

Drop-in for the hot path of MWPainter/Sequential-Variational-Autoencoder: the
unrolled recognition ladder + reparameterised sample + g_theta encoder +
conv-transpose decoder + 16*MSE/KL loss and its backward (sequential_vae.py:877-1212,
1537-1842; abstract_network.py:8-71), behind the reference's
``SequentialVAE.train`` / ``.test`` interface.
"""
from .config import SVAEConfig, PRESETS, preset  # noqa: F401
from . import _lib  # noqa: F401


def __getattr__(name):
    if name == "SequentialVAE":
        from .sequential_vae import SequentialVAE
        return SequentialVAE
    if name == "parallel":
        from . import parallel
        return parallel
    raise AttributeError(name)
