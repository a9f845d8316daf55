"""ctypes loader for the C restatements under oracle/ — TEST INFRASTRUCTURE ONLY (tests/,
__graft_entry__.smoke(), bench.py cpu_baseline).  `make -C oracle` (run by
__graft_entry__.build()) produces oracle/_build/libphc_oracle.so."""

import ctypes
import os

import numpy as np

_LIB = None
_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_build", "libphc_oracle.so")


def lib():
    global _LIB
    if _LIB is None:
        if not os.path.exists(_PATH):
            raise RuntimeError(f"{_PATH} missing: run `make -C oracle`")
        _LIB = ctypes.CDLL(_PATH)
        f = ctypes.POINTER(ctypes.c_float)
        _LIB.phc_oracle_gae.argtypes = [f, f, f, ctypes.c_int64, ctypes.c_float, ctypes.c_float, f]
        _LIB.phc_oracle_gae.restype = None
    return _LIB


def compute_gae(dones, values, rewards, gamma, lam):
    """c_gae.pyx:11-32 in C (float32), same signature as the reference's compute_gae."""
    d, v, r = (np.ascontiguousarray(x, dtype=np.float32) for x in (dones, values, rewards))
    out = np.zeros(len(r), np.float32)
    p = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))  # noqa: E731
    lib().phc_oracle_gae(p(d), p(v), p(r), len(r), float(gamma), float(lam), p(out))
    return out
