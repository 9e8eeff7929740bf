import importlib
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

PKG_NAME = "sequential-variational-autoencoder_amd"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP engine)")
    config.addinivalue_line("markers", "slow: long CPU test")


@pytest.fixture(scope="session")
def pkg():
    return importlib.import_module(PKG_NAME)


def pkg_mod(name):
    return importlib.import_module(PKG_NAME + "." + name)


@pytest.fixture(scope="session")
def built_lib():
    """Build the library (cheap if up to date) so CPU tests can check its ABI."""
    build = pkg_mod("build")
    return build.build()


def gpu_available():
    import torch
    return torch.cuda.is_available()


@pytest.fixture
def knob_lib():
    """Networks created inside the test use the -DSVAE_KNOBS build (libsvae_hip_knobs.so), which reads
    the A/B switches of csrc/knobs.h (SVAE_*) that the shipping library compiles to their defaults."""
    L = pkg_mod("_lib")
    with L.knob_build() as lib:
        yield lib
