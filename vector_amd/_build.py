"""Build libvsig.so in-tree with hipcc for gfx950 (no torch extension machinery:
the library is a plain C-ABI shared object loaded through ctypes)."""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libvsig.so")
SOURCES = ["kernels.hip", "analysis.hip", "pfb.hip", "stream_ops.hip", "vsig_api.hip"]
HEADERS = ["fft_engine.hpp", "vsig_kernels.h"]
ARCH = os.environ.get("VSIG_ARCH", "gfx950")


def _stale() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS]
    deps.append(os.path.join(ROOT, "include", "vsig.h"))
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = True, defines=(), out: str = LIB) -> str:
    """Compile every HIP source into vector_amd/libvsig.so (gfx950).  `defines`
    / `out` build A/B variants (e.g. VSIG_SCALAR_FFT -> libvsig_scalar.so,
    loaded with VSIG_LIB=... by the tuning tools; never by the product)."""
    if out == LIB and not defines and not force and not _stale():
        return LIB
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    tmp = out + ".tmp"
    cmd = [hipcc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-fno-slp-vectorize",   # SLP packs f32 pairs into v_pk_* + v_mov shuffles
           "-Wall", "-Wno-unused-function", *[f"-D{d}" for d in defines],
           *[os.path.join(CSRC, s) for s in SOURCES], "-o", tmp]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, out)
    return out


if __name__ == "__main__":
    if "--scalar" in sys.argv:
        build(defines=("VSIG_SCALAR_FFT",), out=os.path.join(HERE, "libvsig_scalar.so"))
    else:
        build(force="--force" in sys.argv)
