"""ctypes wrapper of oracle/npdot.c -- TEST INFRASTRUCTURE ONLY.

numpy's complex128 np.correlate / np.dot and np.abs restated operation for
operation (OpenBLAS 0.3.29 zdotu order, numpy's SIMD complex abs; see the C
file's header).  Used by tests/test_npdot_cpu.py to pin the restatement against
numpy itself and by the GPU tests as the checker of refine.hip's numpy-order
pass.  Never imported by the product.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "npdot.c")
LIB = os.path.join(HERE, "libnpdot.so")
_lib = None


def build(force: bool = False) -> str:
    """gcc the restatement into oracle/libnpdot.so (no FMA contraction: every
    fma is an explicit fma() call, -mfma makes it the instruction)."""
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(SRC):
        subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-mfma", "-shared", "-fPIC", SRC,
                        "-o", LIB + ".tmp", "-lm"], check=True)
        os.replace(LIB + ".tmp", LIB)
    return LIB


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        lib = C.CDLL(LIB)
        P = C.c_void_p
        lib.np_zdotu.argtypes = [C.c_long, P, P, C.c_long, P]
        lib.np_correlate.argtypes = [P, C.c_long, P, C.c_long, C.c_int, C.c_long, P, P]
        lib.np_cabs.argtypes = [P, C.c_long, P]
        _lib = lib
    return _lib


def _c128(x):
    return np.ascontiguousarray(x, dtype=np.complex128)


def zdotu(x, y, threads: int = 1) -> complex:
    x, y = _c128(x), _c128(y)
    out = np.zeros(2)
    _load().np_zdotu(len(x), x.ctypes.data, y.ctypes.data, threads, out.ctypes.data)
    return complex(out[0], out[1])


def correlate(a, v, mode: str = "full", threads: int = 1) -> np.ndarray:
    a, v = _c128(a), _c128(v)
    na, nv = len(a), len(v)
    n1, n2 = max(na, nv), min(na, nv)
    m = {"valid": 0, "same": 1, "full": 2}[mode]
    length = {0: n1 - n2 + 1, 1: n1, 2: n1 + n2 - 1}[m]
    out = np.zeros(length, np.complex128)
    vc = np.zeros(nv, np.complex128)
    _load().np_correlate(a.ctypes.data, na, v.ctypes.data, nv, m, threads, vc.ctypes.data,
                         out.ctypes.data)
    return out


def cabs(c) -> np.ndarray:
    c = _c128(c)
    out = np.zeros(len(c))
    _load().np_cabs(c.ctypes.data, len(c), out.ctypes.data)
    return out
