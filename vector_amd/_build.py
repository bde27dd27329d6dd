"""Build libvsig.so in-tree with hipcc for gfx950 (no torch extension machinery:
the library is a plain C-ABI shared object loaded through ctypes).  Each HIP
source compiles to its own object in parallel (every kernel is launched from
the translation unit that defines it, so no relocatable device code is
needed), then one link."""
from __future__ import annotations

import hashlib
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libvsig.so")
SOURCES = ["psd.hip", "fir.hip", "xcorr.hip", "reduce.hip", "refine.hip", "bigfft.hip", "analysis.hip", "pfb.hip",
           "stream_ops.hip", "chain.hip", "vsig_api.hip"]
HEADERS = ["fft_engine.hpp", "os_common.hpp", "vsig_kernels.h", "npabs.hpp"]
ARCH = os.environ.get("VSIG_ARCH", "gfx950")


def source_hash() -> str | None:
    """sha256 (16 hex) over the kernel / ABI sources, compiled into the library
    as vsig_build_id() and checked by the loader (None if the sources are not
    next to the package)."""
    h = hashlib.sha256()
    for f in SOURCES + HEADERS:
        p = os.path.join(CSRC, f)
        if not os.path.exists(p):
            return None
        h.update(f.encode())
        h.update(open(p, "rb").read())
    hp = os.path.join(ROOT, "include", "vsig.h")
    if not os.path.exists(hp):
        return None
    h.update(open(hp, "rb").read())
    return h.hexdigest()[:16]


def _stale() -> bool:
    """The library is missing or was built from other sources (its build id,
    recorded next to it at build time, differs from source_hash())."""
    stamp = LIB + ".buildid"
    if not os.path.exists(LIB) or not os.path.exists(stamp):
        return True
    return open(stamp).read().strip() != source_hash()


def build(force: bool = False, verbose: bool = True, defines=(), out: str = LIB) -> str:
    """Compile every HIP source into vector_amd/libvsig.so (gfx950).  `defines`
    / `out` build A/B variants (e.g. VSIG_SCALAR_FFT -> libvsig_scalar.so,
    loaded with VSIG_LIB=... by the tuning tools; never by the product)."""
    if out == LIB and not defines and not force and not _stale():
        return LIB
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
             "-fno-slp-vectorize",   # SLP packs f32 pairs into v_pk_* + v_mov shuffles
             "-Wall", "-Wno-unused-function", f'-DVSIG_SRC_HASH="{source_hash()}"',
             *[f"-D{d}" for d in defines]]
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
    with open(out + ".buildid", "w") as f:
        f.write(source_hash() + "\n")
    return out


if __name__ == "__main__":
    if "--scalar" in sys.argv:
        build(defines=("VSIG_SCALAR_FFT",), out=os.path.join(HERE, "libvsig_scalar.so"))
    elif "--tune" in sys.argv:      # + the engine / copy micro-benchmarks (tools/)
        build(defines=("VSIG_TUNING",), out=os.path.join(HERE, "libvsig_tune.so"))
    else:
        build(force="--force" in sys.argv)
