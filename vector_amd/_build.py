"""Build libvsig.so in-tree with hipcc for gfx950 (no torch extension machinery:
the library is a plain C-ABI shared object loaded through ctypes).  Each HIP
source compiles to its own object in parallel (every kernel is launched from
the translation unit that defines it, so no relocatable device code is
needed), then one link."""
from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libvsig.so")
SOURCES = ["psd.hip", "fir.hip", "xcorr.hip", "reduce.hip", "analysis.hip", "pfb.hip",
           "stream_ops.hip", "firpsd.hip", "vsig_api.hip"]
HEADERS = ["fft_engine.hpp", "os_common.hpp", "vsig_kernels.h"]
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
    flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
             "-fno-slp-vectorize",   # SLP packs f32 pairs into v_pk_* + v_mov shuffles
             "-Wall", "-Wno-unused-function", *[f"-D{d}" for d in defines]]
    objdir = os.path.join(ROOT, "build", os.path.basename(out) + ".obj")
    os.makedirs(objdir, exist_ok=True)

    def compile_one(src):
        obj = os.path.join(objdir, src + ".o")
        cmd = [hipcc, *flags, "-c", os.path.join(CSRC, src), "-o", obj]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
        return obj

    jobs = int(os.environ.get("MAX_JOBS", "0")) or min(len(SOURCES), os.cpu_count() or 1)
    with ThreadPoolExecutor(max_workers=max(1, min(jobs, 16))) as ex:
        objs = list(ex.map(compile_one, SOURCES))
    tmp = out + ".tmp"
    cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", tmp]
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
