"""Build libsvae_hip.so in-tree with hipcc for gfx950 (no cmake needed).

    python sequential-variational-autoencoder_amd/build.py [--force] [--knobs]

Objects go to csrc/build/, the shared library to the package directory, so the
.so travels with a gpurun snapshot (it is git-ignored, not gpurun-ignored).
--knobs builds libsvae_hip_knobs.so (-DSVAE_KNOBS, objects in csrc/build-knobs/): the same
library with the A/B tuning switches of csrc/knobs.h read from the environment; only the
tests that hold an alternative path bitwise to the default and tools/gpu/ab.sh load it.
"""
import hashlib
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


def src_hash():
    """sha256 (16 hex digits) of every source and header the library is compiled from, in a fixed order.
    engine.cpp embeds it (svae_build_hash(), and the literal "SVAE_SRC_HASH=<hash>" in the binary), so
    _lib refuses a library built from other sources and build() skips a library that is already current."""
    h = hashlib.sha256()
    for name in SOURCES + HEADERS:
        with open(os.path.join(CSRC, name), "rb") as f:
            h.update(name.encode() + b"\0" + f.read() + b"\0")
    for name in ("svae_hip.h", "svae_pcnn.h"):
        with open(os.path.join(INCLUDE, name), "rb") as f:
            h.update(name.encode() + b"\0" + f.read() + b"\0")
    return h.hexdigest()[:16]


def embedded_hash(path):
    """The SVAE_SRC_HASH literal a built library carries (None: absent / unreadable)."""
    try:
        with open(path, "rb") as f:
            data = f.read()
    except OSError:
        return None
    i = data.find(b"SVAE_SRC_HASH=")
    return data[i + 14:i + 30].decode("ascii", "replace") if i >= 0 else None


def build(force=False, verbose=False, knobs=False):
    out, extra = (KNOBS_OUT, ["-DSVAE_KNOBS"]) if knobs else (OUT, EXTRA)
    sh = src_hash()
    # a library built from exactly these sources is current whatever the object files' state (they do
    # not travel to the GPU box: the library itself is checked there, and rebuilt only if it is stale)
    if not force and not EXTRA and embedded_hash(out) == sh:
        return out
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
        # engine.cpp carries the source hash: recompiled whenever any source changed
        stale = _mtime(op) < max(_mtime(sp), hdr_t) or (src == "engine.cpp" and embedded_hash(op) != sh)
        if force or stale:
            lang = ["-x", "hip"] if src.endswith(".hip") else []
            defs = ['-DSVAE_SRC_HASH="%s"' % sh] if src == "engine.cpp" else []
            jobs.append([HIPCC] + FLAGS + extra + defs + lang + ["-c", sp, "-o", op])

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
    if jobs or force or _mtime(out) < max(_mtime(o) for o in objs) or embedded_hash(out) != sh:
        run([HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out] + objs)
    return out


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True, knobs="--knobs" in sys.argv))
