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


# objects are cached by (compiler, flags, sources -- the source hash is one of
# the flags): A/B variants that change one translation unit's flags recompile
# only that one
OBJDIR = os.path.join(ROOT, "build", "objcache")


def _compiler(defines=(), src=None):
    """hipcc and its flags for one source (the build id goes into vsig_api.hip
    alone, so an edit elsewhere recompiles only the edited unit and the API)."""
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
             "-fno-slp-vectorize",   # SLP packs f32 pairs into v_pk_* + v_mov shuffles
             "-Wall", "-Wno-unused-function", *[f"-D{d}" for d in defines]]
    if src == "vsig_api.hip":
        flags.append(f'-DVSIG_SRC_HASH="{source_hash()}"')
    return hipcc, flags


def _unit_hash(src: str) -> str:
    """The source and every shared header (any header edit recompiles all)."""
    h = hashlib.sha256()
    for f in [src, *HEADERS]:
        h.update(open(os.path.join(CSRC, f), "rb").read())
    h.update(open(os.path.join(ROOT, "include", "vsig.h"), "rb").read())
    return h.hexdigest()


def object_path(src: str, defines=(), extra=()) -> str:
    """The cached object of one source under these defines / extra flags
    (tests read the product's device code from it: tests/test_isa_cpu.py)."""
    hipcc, flags = _compiler(defines, src)
    key = hashlib.sha256(" ".join([hipcc, *flags, *extra, _unit_hash(src)]).encode()).hexdigest()[:16]
    return os.path.join(OBJDIR, f"{src}.{key}.o")


def compile_object(src: str) -> str:
    """The product object of one source (compiled into the cache if missing)."""
    obj = object_path(src)
    if not os.path.exists(obj):
        hipcc, flags = _compiler((), src)
        os.makedirs(OBJDIR, exist_ok=True)
        subprocess.run([hipcc, *flags, "-c", os.path.join(CSRC, src), "-o", obj + ".tmp"], check=True)
        os.replace(obj + ".tmp", obj)
    return obj


def build(force: bool = False, verbose: bool = True, defines=(), out: str = LIB, src_flags=None) -> str:
    """Compile every HIP source into vector_amd/libvsig.so (gfx950).  `defines`
    / `out` build A/B variants (e.g. VSIG_SCALAR_FFT -> libvsig_scalar.so,
    loaded with VSIG_LIB=... by the tuning tools; never by the product);
    src_flags: {source: [extra compiler flags]} for an A/B of code generation."""
    src_flags = src_flags or {}
    if out == LIB and not defines and not src_flags and not force and not _stale():
        return LIB
    os.makedirs(OBJDIR, exist_ok=True)

    def compile_one(src):
        extra = list(src_flags.get(src, ()))
        obj = object_path(src, defines, extra)
        if os.path.exists(obj) and not force:
            return obj
        hipcc, flags = _compiler(defines, src)
        cmd = [hipcc, *flags, *extra, "-c", os.path.join(CSRC, src), "-o", obj + ".tmp"]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
        os.replace(obj + ".tmp", obj)
        return obj

    jobs = int(os.environ.get("MAX_JOBS", "0")) or min(len(SOURCES), os.cpu_count() or 1)
    with ThreadPoolExecutor(max_workers=max(1, min(jobs, 16))) as ex:
        objs = list(ex.map(compile_one, SOURCES))
    tmp = out + ".tmp"
    hipcc = _compiler()[0]
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
