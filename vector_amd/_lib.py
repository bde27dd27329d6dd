"""ctypes binding of libvsig.so (include/vsig.h) and per-device contexts.

The product path has no CPU fallback: if the library is missing or no HIP
device is present, every compute call raises ``VsigUnavailable``.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

import torch  # loaded first: libvsig.so then binds torch's HIP runtime (same soname)

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libvsig.so")

VSIG_OK = 0
MODES = {"valid": 0, "full": 1, "same": 2}
DTYPES = {"c128": 0, "c64": 1, "f64": 2, "f32": 3}


class VsigUnavailable(RuntimeError):
    """libvsig.so is not built or no HIP device is visible."""


class VsigError(RuntimeError):
    pass


class RefineFault(VsigError):
    """The exact-argmax refine faulted on the device (its watchdog fired,
    vsig.h VSIG_E_REFINE / refine status 3): the peak record is invalid.
    Raised, never warned: the lag / |c| contract is numpy's exact answer."""


class Peak(C.Structure):
    _fields_ = [("peak", C.c_double), ("index", C.c_int64),
                ("sum_abs", C.c_double), ("sum_abs2", C.c_double)]


P = C.c_void_p
I32, I64, F32 = C.c_int32, C.c_int64, C.c_float


class ChainConfig(C.Structure):
    """vsig_chain_config (include/vsig.h)."""
    _fields_ = [("n_local", I64), ("taps", P), ("ntaps", I32), ("decim", I32), ("nfft", I32),
                ("window", P), ("psd_scale", F32), ("tmpl", P), ("L", I64)]


SENDRECV = C.CFUNCTYPE(C.c_int, P, P, I64, I32, P, I64, I32, P)
ALLGATHER = C.CFUNCTYPE(C.c_int, P, P, P, I64, P)


class Transport(C.Structure):
    """vsig_transport (include/vsig.h)."""
    _fields_ = [("user", P), ("sendrecv", SENDRECV), ("allgather", ALLGATHER)]

# name -> (restype, argtypes); every symbol include/vsig.h declares.
SIGNATURES = {
    "vsig_version": (C.c_int, []),
    "vsig_build_id": (C.c_char_p, []),
    "vsig_refine_status": (C.c_int, [P, C.POINTER(I32), C.POINTER(I64)]),
    "vsig_errstr": (C.c_char_p, [C.c_int]),
    "vsig_init": (C.c_int, [C.c_int, C.POINTER(P)]),
    "vsig_free": (None, [P]),
    "vsig_last_error": (C.c_char_p, [P]),
    "vsig_set_stream": (C.c_int, [P, P]),
    "vsig_get_stream": (P, [P]),
    "vsig_copy_dev": (C.c_int, [P, P, P, I64]),
    "vsig_synchronize": (C.c_int, [P]),
    "vsig_set_option": (C.c_int, [P, C.c_char_p, C.c_int]),
    "vsig_get_option": (C.c_int, [P, C.c_char_p, C.POINTER(C.c_int)]),
    "vsig_timing_enable": (C.c_int, [P, C.c_int]),
    "vsig_timing_read": (C.c_int, [P, C.c_char_p, C.POINTER(C.c_double), C.POINTER(I64)]),
    "vsig_timing_reset": (C.c_int, [P]),
    "vsig_clock_enable": (C.c_int, [P, C.c_int]),
    "vsig_refine_stream": (P, [P]),
    "vsig_refine_join": (C.c_int, [P]),
    "vsig_clock_read": (C.c_int, [P, C.c_char_p, C.POINTER(C.c_double), C.POINTER(I64)]),
    "vsig_psd_c64_dev": (C.c_int, [P, P, I64, I64, P, I32, I64, I32, F32, I32, P, I64]),
    "vsig_psd_c64": (C.c_int, [P, P, I64, P, I32, I64, I32, F32, I32, P, I64]),
    "vsig_fir_create": (C.c_int, [P, P, I32, I32, C.POINTER(P)]),
    "vsig_fir_free": (None, [P]),
    "vsig_fir_exec_dev": (C.c_int, [P, P, I64, P, I64]),
    "vsig_fir_exec_hist_dev": (C.c_int, [P, P, I64, I64, P, I64]),
    "vsig_fir_c64": (C.c_int, [P, P, I64, P, I32, I32, P, I64]),
    "vsig_fir_block": (C.c_int, [P]),
    "vsig_fir_exec_mix_dev": (C.c_int, [P, P, I64, I64, P, I64, C.c_double, C.c_double, I64]),
    "vsig_xcorr_create": (C.c_int, [P, P, I64, C.POINTER(P)]),
    "vsig_xcorr_free": (None, [P]),
    "vsig_xcorr_exec_dev": (C.c_int, [P, P, I64, I32, P, P]),
    "vsig_correlate_dev": (C.c_int, [P, I32, P, I64, P, I64, I32, I32, P, P]),
    "vsig_correlate": (C.c_int, [P, I32, P, I64, P, I64, I32, I32, P, P]),
    "vsig_correlate_c64_dev": (C.c_int, [P, P, I64, P, I64, I32, P, P]),
    "vsig_correlate_c64": (C.c_int, [P, P, I64, P, I64, I32, P, P]),
    "vsig_dft_dev": (C.c_int, [P, I32, P, I64, I64, I32, I32, P]),
    "vsig_resample_dev": (C.c_int, [P, I32, P, I64, I64, I32, P]),
    "vsig_filter_channel_dev": (C.c_int, [P, I32, P, I64, C.c_double, C.c_double, C.c_double, P]),
    "vsig_peak_dev": (C.c_int, [P, I32, P, I64, P]),
    "vsig_peak": (C.c_int, [P, I32, P, I64, P]),
    "vsig_abs_stats_dev": (C.c_int, [P, I32, P, I64, P]),
    "vsig_correlate_stats_dev": (C.c_int, [P, I32, P, I64, P, I64, I32, P]),
    "vsig_mix_c64_dev": (C.c_int, [P, P, I64, C.c_double, C.c_double, I64, P]),
    "vsig_scale_c64_dev": (C.c_int, [P, P, I64, C.c_float, P]),
    "vsig_wv_quantize_dev": (C.c_int, [P, P, I64, C.c_float, P]),
    "vsig_planar_to_c64_dev": (C.c_int, [P, I32, P, P, I64, P]),
    "vsig_c64_to_planar_dev": (C.c_int, [P, P, I64, P, P]),
    "vsig_pfb_c64_dev": (C.c_int, [P, P, I64, P, I32, I32, P, I64]),
    "vsig_select_dev": (C.c_int, [P, I32, P, I64, C.POINTER(I64), I32, C.POINTER(C.c_double)]),
    "vsig_threshold_dev": (C.c_int, [P, I32, P, I64, C.c_double, C.POINTER(I64), C.POINTER(I64),
                                     C.POINTER(I64), C.POINTER(C.c_double)]),
    "vsig_boxcar_energy_dev": (C.c_int, [P, I32, P, I64, I64, P]),
    "vsig_db_dev": (C.c_int, [P, I32, P, I64, C.c_double, P]),
    "vsig_abs_c64_dev": (C.c_int, [P, I32, P, I64, P]),
    "vsig_abs_c128_dev": (C.c_int, [P, I32, P, I64, P]),
    "vsig_chain_create": (C.c_int, [P, C.POINTER(ChainConfig), I32, I32, C.POINTER(Transport),
                                    C.POINTER(P)]),
    "vsig_chain_free": (None, [P]),
    "vsig_chain_last_error": (C.c_char_p, [P]),
    "vsig_chain_input": (P, [P]),
    "vsig_chain_step": (C.c_int, [P]),
    "vsig_chain_result": (C.c_int, [P, C.POINTER(Peak), C.POINTER(I64)]),
    "vsig_chain_filtered": (P, [P, C.POINTER(I64)]),
    "vsig_chain_spectra": (P, [P, C.POINTER(I64)]),
    "vsig_rccl_available": (C.c_int, []),
    "vsig_rccl_unique_id": (C.c_int, [C.c_char_p]),
    "vsig_rccl_comm_init": (C.c_int, [I32, I32, C.c_char_p, I32, C.POINTER(P)]),
    "vsig_rccl_comm_destroy": (C.c_int, [P]),
    "vsig_rccl_transport": (C.c_int, [P, C.POINTER(Transport)]),
    "vsig_loopback_create": (C.c_int, [I32, C.POINTER(P)]),
    "vsig_loopback_free": (None, [P]),
    "vsig_loopback_transport": (C.c_int, [P, I32, C.POINTER(Transport)]),
}

_lib = None
_lib_lock = threading.Lock()


def load_library(path: str | None = None):
    """Load libvsig.so and declare every entry point; no device needed.
    (VSIG_LIB selects an A/B build of the same sources, for the tuning tools.)
    The library's build id must equal the hash of the kernel sources next to
    it (vector_amd/csrc, include/vsig.h): a stale binary is refused."""
    global _lib
    path = path or os.environ.get("VSIG_LIB") or LIB_PATH
    with _lib_lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise VsigUnavailable(
                f"{path} is not built: run `python -c 'import __graft_entry__ as g; g.build()'` "
                "(hipcc --offload-arch=gfx950)")
        lib = C.CDLL(path)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        from ._build import source_hash
        want, got = source_hash(), lib.vsig_build_id().decode()
        if want is not None and got != want:
            raise VsigUnavailable(f"{path} was built from other sources (build id {got}, sources "
                                  f"{want}): rebuild with `python -m vector_amd._build`")
        _lib = lib
        return lib


_warned_no_threadpoolctl = False
_blas_ctl = None            # threadpoolctl controller of numpy's OpenBLAS (found once)


def numpy_blas_threads() -> int:
    """The thread count of the OpenBLAS behind this process's numpy (its zdotu
    splits a complex128 dot of more than 10000 terms into that many chunks,
    which decides the rounding of np.correlate's long sums); read at every call
    (threadpool_limits / OPENBLAS_NUM_THREADS may change it) through a
    controller found once (threadpool_info() rescans every loaded library:
    ~5 ms a call; the controller's get_num_threads is one C call into
    OpenBLAS).  1 if unknown -- with a warning when threadpoolctl is missing:
    correlations with more than 10000 overlap terms then match numpy only if
    its OpenBLAS runs one thread."""
    global _warned_no_threadpoolctl, _blas_ctl
    if _blas_ctl is None:
        try:
            import numpy  # noqa: F401  (its OpenBLAS is loaded with it)
            from threadpoolctl import ThreadpoolController
        except ImportError:
            if not _warned_no_threadpoolctl:
                import warnings
                warnings.warn("threadpoolctl is not importable: numpy's OpenBLAS thread count is "
                              "taken as 1 for the exact argmax of correlations over 10000 terms",
                              RuntimeWarning, stacklevel=2)
                _warned_no_threadpoolctl = True
            return 1
        try:
            ctl = [lc for lc in ThreadpoolController().lib_controllers if lc.internal_api == "openblas"]
        except Exception:
            ctl = []
        _blas_ctl = ctl[0] if ctl else False
    if not _blas_ctl:
        return 1
    try:
        return max(1, min(1024, int(_blas_ctl.get_num_threads())))
    except Exception:
        return 1


class Context:
    """One vsig_ctx on one device (the library's stream state lives here)."""

    def __init__(self, device: int):
        lib = load_library()
        h = P()
        rc = lib.vsig_init(device, C.byref(h))
        if rc != VSIG_OK:
            raise VsigUnavailable(f"vsig_init(device={device}) failed: "
                                  f"{lib.vsig_errstr(rc).decode()}")
        self.lib, self.h, self.device = lib, h, device
        self.blas_threads = None
        self.sync_blas_threads()

    def sync_blas_threads(self):
        """The refine matches numpy's complex128 sums operation for operation;
        OpenBLAS splits those over 10000 terms across its threads: hand the
        library numpy's current thread count (called before each correlation)."""
        t = numpy_blas_threads()
        if t != self.blas_threads:
            self.check(self.lib.vsig_set_option(self.h, b"blas_threads", t), "blas_threads")
            self.blas_threads = t

    def check(self, rc: int, what: str):
        if rc != VSIG_OK:
            msg = self.lib.vsig_last_error(self.h).decode()
            err = self.lib.vsig_errstr(rc).decode()
            if rc == -1:
                raise ValueError(f"{what}: {err}: {msg}")
            if rc == -4:
                raise NotImplementedError(f"{what}: {err}: {msg}")
            if rc == -6:
                raise RefineFault(f"{what}: {err}: {msg}")
            raise VsigError(f"{what}: {err}: {msg}")

    def bind_stream(self):
        """Enqueue on torch's current stream (so torch events time our kernels)."""
        s = torch.cuda.current_stream(self.device).cuda_stream
        self.check(self.lib.vsig_set_stream(self.h, P(s)), "vsig_set_stream")

    def __del__(self):
        try:
            if self.h:
                self.lib.vsig_free(self.h)
                self.h = None
        except Exception:
            pass


_ctx_tls = threading.local()


def get_context(device: int | None = None) -> Context:
    """Per-thread, per-device context bound to torch's current stream."""
    if not torch.cuda.is_available():
        raise VsigUnavailable("vector_amd needs a HIP device (torch.cuda.is_available() is False); "
                              "there is no CPU fallback")
    if device is None:
        device = torch.cuda.current_device()
    cache = getattr(_ctx_tls, "ctx", None)
    if cache is None:
        cache = _ctx_tls.ctx = {}
    ctx = cache.get(device)
    if ctx is None:
        with torch.cuda.device(device):
            ctx = cache[device] = Context(device)
    ctx.bind_stream()
    return ctx
