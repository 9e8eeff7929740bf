"""Parameter table + deterministic initialisation of the flat parameter buffer.

The table (names, TF shapes, offsets) comes from the library (``svae_param_layout``)
so the host and the engine can never disagree.  Initial values follow the
reference initialisers (abstract_network.py:19,38,47,57,66: N(0, 0.02); default
xavier-uniform for the heads / output conv-T, sequential_vae.py:1592-1609,1720,1727;
zero biases and BN beta) drawn from a counter-based splitmix64 stream keyed by
(seed, tensor name), so any implementation can regenerate them bit-exactly.
"""
import ctypes

import numpy as np

from . import _lib

INIT_NAMES = {0: "zeros", 1: "normal0.02", 2: "glorot"}
FLAG_DEAD, FLAG_ZERO_GRAD = 1, 2

_G = 0x9E3779B97F4A7C15
_MASK = (1 << 64) - 1


def param_table(cfg):
    L = _lib.lib()
    c = cfg.to_c()
    nt, nl, n = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int32()
    _lib.check(L.svae_param_count(ctypes.byref(c), ctypes.byref(nt), ctypes.byref(nl), ctypes.byref(n)))
    arr = (_lib.SvaeParamDesc * n.value)()
    _lib.check(L.svae_param_layout(ctypes.byref(c), arr, n.value))
    table = []
    for d in arr:
        shape = tuple(int(d.shape[i]) for i in range(d.ndim))
        table.append(dict(name=d.name.decode(), shape=shape, offset=int(d.offset), size=int(np.prod(shape)),
                          init=INIT_NAMES[d.init], dead=bool(d.flags & FLAG_DEAD),
                          zero_grad=bool(d.flags & FLAG_ZERO_GRAD)))
    return table, int(nt.value), int(nl.value)


def _name_key(name):
    h = 0xCBF29CE484222325
    for b in name.encode("utf-8"):
        h = ((h ^ b) * 0x100000001B3) & _MASK
    return h


def _uniform(name, seed, n):
    key = np.uint64(_name_key(name) ^ ((seed * _G) & _MASK))
    with np.errstate(over="ignore"):
        z = np.arange(1, n + 1, dtype=np.uint64) * np.uint64(_G) + key
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return (z >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


def init_value(name, shape, init, seed):
    n = int(np.prod(shape))
    if init == "zeros":
        return np.zeros(n)
    if init == "normal0.02":
        m = (n + 1) // 2
        u = _uniform(name, seed, 2 * m)
        r = np.sqrt(-2.0 * np.log1p(-u[0::2]))
        th = 2.0 * np.pi * u[1::2]
        v = np.empty(2 * m)
        v[0::2], v[1::2] = r * np.cos(th), r * np.sin(th)
        return 0.02 * v[:n]
    if init == "glorot":
        if len(shape) == 2:
            fi, fo = shape
        else:
            rf = int(np.prod(shape[:-2]))
            fi, fo = shape[-2] * rf, shape[-1] * rf
        return (2.0 * _uniform(name, seed, n) - 1.0) * np.sqrt(6.0 / (fi + fo))
    raise ValueError(init)


def init_flat(cfg, seed=0):
    """Flat fp32 host buffer with every tensor at its layout offset."""
    table, n_total, _ = param_table(cfg)
    flat = np.zeros(n_total, dtype=np.float32)
    for p in table:
        flat[p["offset"]:p["offset"] + p["size"]] = init_value(p["name"], p["shape"], p["init"], seed)
    return flat


def unflatten(flat, table):
    """name -> array view in TF shape."""
    return {p["name"]: np.asarray(flat[p["offset"]:p["offset"] + p["size"]]).reshape(p["shape"]) for p in table}
