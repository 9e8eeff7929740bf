"""The shipping library reads no environment (csrc/knobs.h).

Every A/B tuning switch compiles to its default in libsvae_hip.so; only libsvae_hip_knobs.so
(-DSVAE_KNOBS) reads SVAE_* variables, and the timing probe SVAE_DBG_SKIP (deliberately wrong
results) exists only in a -DSVAE_DEBUG_PROBES build.  The CPU tests check the sources and the
built library's imports; the GPU test runs a training step with every probe bit set in the
environment and holds it bitwise to the step without."""
import glob
import json
import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "sequential-variational-autoencoder_amd", "csrc")


def test_sources_read_at_most_ten_variables():
    n = 0
    for f in glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp")) + \
            glob.glob(os.path.join(CSRC, "*.h")):
        src = open(f).read()
        n += len(re.findall(r"\bgetenv\s*\(", src))
    assert n <= 10, n


def test_default_library_imports_no_getenv(built_lib):
    out = subprocess.run(["nm", "-D", "--undefined-only", built_lib], capture_output=True, text=True).stdout
    assert not re.search(r"\bgetenv\b", out), "libsvae_hip.so imports getenv"
    assert b"SVAE_DBG_SKIP" not in open(built_lib, "rb").read()


_STEP = r'''
import hashlib, json, sys
sys.path.insert(0, %r)
import importlib, torch
cfgmod = importlib.import_module("sequential-variational-autoencoder_amd.config")
SV = importlib.import_module("sequential-variational-autoencoder_amd.sequential_vae").SequentialVAE
from oracle import spec
net = SV(cfgmod.preset("tiny", batch=4, dtype="bf16"), seed=0)
cd = spec.make_config("tiny", batch=4)
x, tgt, eps = spec.make_inputs(cd, batch=4)
for it in (1, 2):
    net.forward(x, tgt, eps, 1.0)
    net.backward_apply(2e-4, it)
torch.cuda.synchronize()
print(json.dumps({"loss": net.loss_value(), "params": hashlib.sha256(net.params.cpu().numpy().tobytes()).hexdigest()}))
'''


@pytest.mark.gpu
def test_debug_probe_variable_has_no_effect():
    outs = []
    for probe in (None, "31"):
        env = dict(os.environ)
        env.pop("SVAE_DBG_SKIP", None)
        if probe:
            env["SVAE_DBG_SKIP"] = probe
        r = subprocess.run([sys.executable, "-c", _STEP % ROOT], cwd=ROOT, env=env, capture_output=True, text=True,
                           timeout=300)
        assert r.returncode == 0, r.stderr[-3000:]
        outs.append(json.loads(r.stdout.strip().splitlines()[-1]))
    assert outs[0] == outs[1], outs
