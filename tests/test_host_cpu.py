"""CPU-only checks of the product's host side: the C-ABI library loads and
exports every symbol include/vsig.h declares, the host parameter logic matches
the reference's recorded calls, windows match scipy, and compute calls fail
loudly (no CPU fallback) when there is no HIP device."""
import os
import re

import numpy as np
import pytest
import scipy.signal

from conftest import ROOT, golden


def header_functions():
    txt = open(os.path.join(ROOT, "include", "vsig.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(vsig_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    from vector_amd import _lib
    lib = _lib.load_library()
    names = header_functions()
    assert len(names) >= 20
    for n in names:
        assert hasattr(lib, n), n
    assert set(names) == set(_lib.SIGNATURES), "ctypes signatures out of sync with vsig.h"
    assert lib.vsig_version() >= 1
    assert lib.vsig_errstr(-4) == b"unsupported size"


def test_library_is_gfx950_code_object():
    so = os.path.join(ROOT, "vector_amd", "libvsig.so")
    blob = open(so, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob        # offload bundle target id


def test_init_without_device_reports_nodevice():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a device is present")
    import ctypes as C
    from vector_amd import _lib
    lib = _lib.load_library()
    h = C.c_void_p()
    assert lib.vsig_init(0, C.byref(h)) == -5      # VSIG_E_NODEVICE


def test_compute_fails_loudly_without_device():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a device is present")
    import vector_amd as va
    x = np.ones(4096, np.complex64)
    for call in (lambda: va.spectrum(x, 1.0, "hann", 256),
                 lambda: va.filter(x, np.ones(8)),
                 lambda: va.cross_correlate_signals(x[:16], x),
                 lambda: va.create_spectrogram(x, 56e6)):
        with pytest.raises(va.VsigUnavailable):
            call()


def test_spectrogram_params_match_reference_calls():
    from vector_amd.spectrogram import spectrogram_params
    g = golden("spec_params.npz")
    cols = list(g["columns"])
    for row in g["table"]:
        r = dict(zip(cols, row))
        p = spectrogram_params(int(r["n"]), r["sr"], int(r["max_samples"]), r["time_res_us"],
                               bool(r["adaptive"]))
        assert (p["nsig"], p["nperseg"], p["noverlap"], p["nfft"]) == \
            (r["nsig"], r["nperseg"], r["noverlap"], r["nfft"])
        assert p["fs"] == pytest.approx(r["fs"], rel=1e-15)
        assert (p["window"] == "hann") == bool(r["window_is_hann"])
    with pytest.raises(ValueError, match="Signal is empty"):
        spectrogram_params(0, 1.0)


@pytest.mark.parametrize("name", ["hann", "hamming", "blackman", "blackmanharris", "nuttall",
                                  "flattop", "boxcar", "bartlett", "triang", ("kaiser", 8.6)])
@pytest.mark.parametrize("n", [1, 2, 31, 32, 560, 1024, 8192])
def test_windows_match_scipy(name, n):
    from vector_amd.windows import get_window
    np.testing.assert_allclose(get_window(name, n), scipy.signal.get_window(name, n),
                               rtol=0, atol=2e-15)


def test_lag_axes_and_lengths():
    from vector_amd.dsp import _corr_len, _lags
    from oracle.ref import cross_correlate_signals
    rng = np.random.default_rng(1)
    for l1, l2 in ((7, 20), (8, 20), (20, 7), (5, 5), (1, 9)):
        s1 = rng.standard_normal(l1) + 0j
        s2 = rng.standard_normal(l2) + 0j
        for mode in ("full", "valid", "same"):
            c, lags = cross_correlate_signals(s1, s2, mode)
            np.testing.assert_array_equal(_lags(mode, l1, l2), lags)
            assert _corr_len(mode, l2, l1) == len(c)


def test_confidence_formula():
    from vector_amd.dsp import _confidence
    rng = np.random.default_rng(2)
    a = np.abs(rng.standard_normal(1000) + 1j * rng.standard_normal(1000))
    a[17] = 40.0
    want = np.clip((a.max() - a.mean()) / a.std() / 10, 0, 1)
    got = _confidence(a.max(), a.sum(), (a * a).sum(), a.size, 0.5)
    assert got == pytest.approx(want, abs=1e-12)
    assert _confidence(1.0, 10.0, 10.0, 10, 0.5) == 0.0          # flat |c|
    assert _confidence(a.max(), a.sum(), (a * a).sum(), a.size, 1.5) == 0.0


def test_correlate_offsets_model():
    """The C layer's (F, nout, off) for np.correlate modes, checked in numpy:
    c[o] = sum_k s[o - off + k] conj(p[k]) with the shorter operand as p."""
    rng = np.random.default_rng(3)

    def model(a, v, mode):
        na, nv = len(a), len(v)
        nmin, nmax = min(na, nv), max(na, nv)
        F, nout = {"full": (0, na + nv - 1), "valid": (nmin - 1, nmax - nmin + 1),
                   "same": ((nmin - 1 - nmin // 2) if na >= nv else nmin // 2, nmax)}[mode]
        swap = nv > na
        p, s = (a, v) if swap else (v, a)
        L = nmin
        off = F + nout - nv if swap else (L - 1) - F
        c = np.zeros(nout, complex)
        for o in range(nout):
            acc = 0j
            for k in range(L):
                i = o - off + k
                if 0 <= i < nmax:
                    acc += s[i] * np.conj(p[k])
            c[o] = acc
        return np.conj(c[::-1]) if swap else c

    for na, nv in ((20, 7), (20, 8), (7, 20), (8, 20), (5, 5), (1, 4), (4, 1)):
        a = rng.standard_normal(na) + 1j * rng.standard_normal(na)
        v = rng.standard_normal(nv) + 1j * rng.standard_normal(nv)
        for mode in ("full", "valid", "same"):
            np.testing.assert_allclose(model(a, v, mode), np.correlate(a, v, mode), atol=1e-12)


def _build_c_example(out, name="chain_c"):
    import shutil
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lib = os.path.join(root, "vector_amd", "libvsig.so")
    if shutil.which("gcc") is None or not os.path.exists(lib):
        pytest.skip("gcc or libvsig.so missing")
    cmd = ["gcc", "-std=c99", "-O2", "-Wall", "-Werror", "-I", os.path.join(root, "include"),
           os.path.join(root, "examples", name + ".c"), "-L", os.path.dirname(lib), "-lvsig",
           f"-Wl,-rpath,{os.path.dirname(lib)}", "-lpthread", "-lm", "-o", out]
    subprocess.run(cmd, check=True)
    return out


@pytest.mark.parametrize("name", ["chain_c", "shard_c"])
def test_c_examples_compile(tmp_path, name):
    """include/vsig.h is plain C99 and the examples (the chain; the sharded
    chain over the loopback / RCCL transports) link against the library's
    exported symbols (the non-Python binding of INTEGRATION.md)."""
    assert os.path.exists(_build_c_example(str(tmp_path / name), name))


def test_numpy_blas_threads_tracks_limits():
    """The refine's OpenBLAS thread count follows threadpool_limits at every
    call, through a controller found once (no per-call library rescan: ADVICE
    r04 -- threadpool_info() costs milliseconds)."""
    import time
    from threadpoolctl import threadpool_info, threadpool_limits
    from vector_amd._lib import numpy_blas_threads
    want = [d["num_threads"] for d in threadpool_info() if d.get("internal_api") == "openblas"]
    if not want:
        pytest.skip("numpy without OpenBLAS")
    assert numpy_blas_threads() == want[0]
    with threadpool_limits(1):
        assert numpy_blas_threads() == 1
    assert numpy_blas_threads() == want[0]
    t0 = time.perf_counter()
    for _ in range(200):
        numpy_blas_threads()
    assert (time.perf_counter() - t0) / 200 < 1e-3


def test_bench_practical_ceiling_uses_newest_probe():
    """bench.py's practical_peak comes from the newest committed membw probe,
    the 4:1 pattern over every variant of it (profiles/r05_membw.json)."""
    import bench
    pc = bench.practical_ceiling("read4to1")
    assert pc is not None and "r05_membw.json" in pc[1]
    import json
    d = json.load(open(os.path.join(ROOT, "profiles", "r05_membw.json")))
    best = max(v[1] for k, v in d.items() if k.startswith(("read4to1", "r4w")))
    assert pc[0] == best and best > 6000
    cp = bench.practical_ceiling("copy")
    assert cp is not None and cp[0] > 6000
