"""Tuning-build loader for tools/: libvsig_tune.so (python -m vector_amd._build
--tune) = the product sources + VSIG_TUNING (the FFT-engine and copy
micro-benchmarks).  Import before vector_amd; never used by the product."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("VSIG_LIB", os.path.join(ROOT, "vector_amd", "libvsig_tune.so"))

from vector_amd import _lib  # noqa: E402

_lib.SIGNATURES.update({
    "vsig_copy_bench": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_int, C.c_int]),
    "vsig_fft_bench": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_int]),
})
