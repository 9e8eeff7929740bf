"""Build libsvae_hip.so in-tree with hipcc for gfx950 (no cmake needed).

    python sequential-variational-autoencoder_amd/build.py [--force] [--knobs]

Objects go to csrc/build/, the shared library to the package directory, so the
.so travels with a gpurun snapshot (it is git-ignored, not gpurun-ignored).
--knobs builds libsvae_hip_knobs.so (-DSVAE_KNOBS, objects in csrc/build-knobs/): the same
library with the A/B tuning switches of csrc/knobs.h read from the environment; only the
tests that hold an alternative path bitwise to the default and tools/gpu/ab.sh load it.
"""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
INCLUDE = os.path.join(os.path.dirname(HERE), "include")
OUT = os.path.join(HERE, "libsvae_hip.so")
SOURCES = ["gemm.hip", "gemm_bf16.hip", "wgrad_halo2.hip", "wgrad_smallc.hip", "smallc.hip", "bn.hip", "misc.hip", "chain.hip", "halo_kw.hip", "halo_x3.hip", "dense_kw.hip", "pcnn.hip", "engine.cpp"]
HEADERS = ["common.h", "kernels.h", "knobs.h", "opload.h"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-mcode-object-version=5",
         "-I" + INCLUDE, "-I" + CSRC, "-Wno-unused-result"]
# A/B builds of compile-time variants: SVAE_CFLAGS="-DSVAE_WT=1" SVAE_BUILD_OUT=ab/wt.so (objects in
# csrc/build-<name>); the default build ignores both
EXTRA = os.environ.get("SVAE_CFLAGS", "").split()
if os.environ.get("SVAE_BUILD_OUT"):
    OUT = os.path.abspath(os.environ["SVAE_BUILD_OUT"])
KNOBS_OUT = os.path.join(HERE, "libsvae_hip_knobs.so")


def _mtime(p):
    return os.path.getmtime(p) if os.path.exists(p) else 0.0


def build(force=False, verbose=False, knobs=False):
    out, extra = (KNOBS_OUT, ["-DSVAE_KNOBS"]) if knobs else (OUT, EXTRA)
    bdir = os.path.join(CSRC, "build" if out.endswith("libsvae_hip.so") and not extra
                        else "build-" + os.path.splitext(os.path.basename(out))[0].replace("libsvae_hip_", ""))
    os.makedirs(bdir, exist_ok=True)
    hdr_t = max(_mtime(os.path.join(CSRC, h)) for h in HEADERS)
    hdr_t = max(hdr_t, _mtime(os.path.join(INCLUDE, "svae_hip.h")), _mtime(os.path.join(INCLUDE, "svae_pcnn.h")))
    jobs = []
    objs = []
    for src in SOURCES:
        sp = os.path.join(CSRC, src)
        op = os.path.join(bdir, os.path.splitext(src)[0] + ".o")
        objs.append(op)
        if force or _mtime(op) < max(_mtime(sp), hdr_t):
            lang = ["-x", "hip"] if src.endswith(".hip") else []
            jobs.append([HIPCC] + FLAGS + extra + lang + ["-c", sp, "-o", op])

    def run(cmd):
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("hipcc failed:\n%s\n%s" % (" ".join(cmd), r.stderr[-4000:]))
        return r

    if jobs:
        with ThreadPoolExecutor(max_workers=min(len(jobs), 8)) as ex:
            list(ex.map(run, jobs))
    if jobs or force or _mtime(out) < max(_mtime(o) for o in objs):
        run([HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out] + objs)
    return out


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True, knobs="--knobs" in sys.argv))
