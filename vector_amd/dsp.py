"""Python front end of the hot path — the reference's call signatures, the
MI355X kernels underneath (libvsig.so through ctypes, no CPU fallback).

Reference functions mirrored (ramiyako/vector utils.py):
  create_spectrogram        utils.py:161-353  (parameter logic restated in spectrogram.py)
  cross_correlate_signals   utils.py:1258-1295
  find_correlation_peak     utils.py:1298-1342
  find_packet_location_in_vector  utils.py:1372-1434
and the north-star front-end names:
  spectrum(x, fs, window, nperseg, noverlap, nfft)  == scipy.signal.spectrogram as called
                                                       at utils.py:281-291
  filter(x, taps, decim)    == np.convolve(x, taps, 'full')[:len(x)][::decim]
  correlate(signal1, signal2, mode) == cross_correlate_signals
  correlate_peak(...)       == find_correlation_peak(*correlate(...)) fused on the GPU

Inputs may be numpy arrays (results come back as numpy, with the reference's
dtypes) or CUDA torch tensors (results stay on the device, fp32/complex64,
nothing is synchronised).  Every computation runs in the HIP kernels.
"""
from __future__ import annotations

import ctypes as C
import warnings
from collections import OrderedDict

import numpy as np
import torch

from . import _lib
from .windows import get_window

__all__ = ["spectrum", "filter", "fir_filter", "correlate", "correlate_peak",
           "cross_correlate_signals", "find_correlation_peak",
           "find_packet_location_in_vector", "FirFilter", "Correlator", "peak_stats",
           "refine_status", "check_refine"]

PEAK_BYTES = 32  # sizeof(vsig_peak_t)


# ---------------------------------------------------------------------------
# helpers
# ---------------------------------------------------------------------------
def _is_dev(x) -> bool:
    return isinstance(x, torch.Tensor)


def _device_c64(x, ctx):
    """1-D complex64 contiguous CUDA tensor of x (host arrays are uploaded)."""
    if _is_dev(x):
        t = x
        if t.dim() != 1:
            raise ValueError("vector_amd works on 1-D signals")
        if not t.is_cuda:
            t = t.to(f"cuda:{ctx.device}")
        if t.dtype != torch.complex64:
            t = t.to(torch.complex64)
        return t.contiguous()
    a = np.asarray(x)
    if a.ndim != 1:
        raise ValueError("vector_amd works on 1-D signals")
    a = np.ascontiguousarray(a, dtype=np.complex64)
    return torch.from_numpy(a).to(f"cuda:{ctx.device}")


def _ptr(t: torch.Tensor):
    return C.c_void_p(t.data_ptr())


def _check_dev(t: torch.Tensor, n: int, dtype, what: str, device=None):
    """Host-side shape check before a kernel writes / reads a caller buffer."""
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise ValueError(f"{what}: expected a CUDA tensor")
    if t.dtype != dtype:
        raise ValueError(f"{what}: dtype {t.dtype}, expected {dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{what}: must be contiguous")
    if t.numel() < n:
        raise ValueError(f"{what}: {t.numel()} elements, need {n}")
    if device is not None and t.device.index != device:
        raise ValueError(f"{what}: on {t.device}, expected cuda:{device}")


def _peak_buffer(ctx):
    return torch.empty(PEAK_BYTES // 8, dtype=torch.float64, device=f"cuda:{ctx.device}")


def _read_peak(buf: torch.Tensor):
    """(max, index, sum_abs, sum_abs2) from a device vsig_peak_t."""
    h = buf.cpu()
    raw = h.numpy()
    idx = int(h.view(torch.int64)[1].item())
    return float(raw[0]), idx, float(raw[2]), float(raw[3])


def _confidence_np(peak, mean, std, threshold_ratio):
    """find_correlation_peak's confidence (utils.py:1328-1340) from numpy's
    mean_corr / std_corr, with the reference's arithmetic."""
    if std > 0:
        conf = np.clip(((np.float64(peak) - mean) / std) / 10.0, 0.0, 1.0)
    else:
        conf = 0.0
    if peak < threshold_ratio * peak:   # utils.py:1339: peak == max(|c|)
        conf = 0.0
    return conf


# The fused correlators sum fp32 |c| values; their single-pass variance
# var = s2/n - mean^2 carries the sums' relative error e (~1e-7: fp32 FFT
# outputs, fp32 per-thread sums, double beyond) amplified by (s2/n) / var.
# Above _FUSED_VAR_FLOOR of the mean square the amplification is <= 20 and the
# std is within ~1e-6 of numpy's (confidence to the 1e-5 bar, tests); below it
# -- a flat |c| (a tone: std of rounding noise), or a tone under weak noise --
# the statistics are recomputed from numpy-order values
# (vsig_correlate_stats_dev: every output re-evaluated as np.correlate forms
# it, then numpy's two-pass mean / std).  Rayleigh-like |c| of noise sits at
# var / (s2/n) = 1 - pi/4 = 0.21 and keeps the fused sums.
_FUSED_VAR_FLOOR = 0.05


def _fused_stats(peak, s1, s2, n):
    """(mean, std, resolved) from the fused record's sums."""
    mean = s1 / n
    ms = s2 / n
    var = ms - mean * mean
    std = float(np.sqrt(var)) if var > 0 else 0.0
    return mean, std, var > _FUSED_VAR_FLOOR * ms


def _confidence(peak, s1, s2, n, threshold_ratio):
    """The confidence from a fused record's sums (single pass; see _FUSED_VAR_FLOOR)."""
    mean, std, _ = _fused_stats(peak, s1, s2, n)
    return _confidence_np(peak, mean, std, threshold_ratio)


def _abs_stats(t: torch.Tensor, code: str, ctx):
    """numpy's (np.mean, np.std) of |t| on the GPU (vsig_abs_stats_dev)."""
    out = torch.empty(2, dtype=torch.float64, device=t.device)
    ctx.check(ctx.lib.vsig_abs_stats_dev(ctx.h, _lib.DTYPES[code], _ptr(t), int(t.numel()), _ptr(out)),
              "abs stats")
    m, sd = out.cpu().tolist()
    return np.float64(m), np.float64(sd)


# ---------------------------------------------------------------------------
# spectrum — scipy.signal.spectrogram(..., return_onesided=False, detrend=False,
# scaling='spectrum') (utils.py:281-291)
# ---------------------------------------------------------------------------
def _triage(window, nperseg, n):
    """scipy.signal._spectral_py._triage_segments for a 1-D input of length n."""
    if isinstance(window, (str, tuple)):
        if nperseg is None:
            nperseg = 256
        if nperseg > n:
            warnings.warn(f"nperseg = {nperseg:d} is greater than input length  = {n:d}, "
                          f"using nperseg = {n:d}", stacklevel=3)
            nperseg = n
        win = get_window(window, nperseg)
    else:
        win = np.asarray(window)
        if win.ndim != 1:
            raise ValueError("window must be 1-D")
        if n < win.shape[-1]:
            raise ValueError("window is longer than input signal")
        if nperseg is None:
            nperseg = win.shape[0]
        elif nperseg != win.shape[0]:
            raise ValueError("value specified for nperseg is different from length of window")
    return win, int(nperseg)


def _out_real_dtype(x):
    dt = x.dtype if not _is_dev(x) else None
    if dt is None:
        return None
    return np.float64 if np.result_type(dt, np.complex64) == np.complex128 else np.float32


def spectrum(x, fs=1.0, window="hann", nperseg=None, noverlap=None, nfft=None, *,
             fftshift=False, _stride=1, _nsamples=None):
    """(f, t, Sxx) of ``scipy.signal.spectrogram(x, fs, window, nperseg, noverlap,
    nfft, detrend=False, return_onesided=False, scaling='spectrum')``.

    Sxx has shape (nfft, nframes) (a transposed view of the frame-major output
    the kernel writes, like scipy's own strided result).  fftshift=True
    returns Sxx already np.fft.fftshift-ed along frequency (f is not shifted).
    """
    if _is_dev(x):
        n = int(_nsamples if _nsamples is not None else x.shape[0])
    else:
        x = np.asarray(x)
        if x.ndim != 1:
            raise ValueError("vector_amd works on 1-D signals")
        n = x.shape[0]
    if n == 0:
        e = np.empty((0,))
        return e, e, e
    win, nperseg = _triage(window, nperseg, n)
    if nfft is None:
        nfft = nperseg
    elif nfft < nperseg:
        raise ValueError("nfft must be greater than or equal to nperseg.")
    nfft = int(nfft)
    noverlap = nperseg // 2 if noverlap is None else int(noverlap)
    if noverlap >= nperseg:
        raise ValueError("noverlap must be less than nperseg.")
    hop = nperseg - noverlap
    nframes = (n - nperseg) // hop + 1
    win32 = win.astype(np.float32)
    scale = float(1.0 / float(np.sum(win32, dtype=np.float64)) ** 2)

    ctx = _lib.get_context()
    dev = f"cuda:{ctx.device}"
    if _is_dev(x):
        xd = x if x.dtype == torch.complex64 else x.to(torch.complex64)
        if not xd.is_contiguous():
            xd = xd.contiguous()
    else:
        xd = _device_c64(x, ctx)
    wd = torch.from_numpy(win32).to(dev)
    out = torch.empty((nframes, nfft), dtype=torch.float32, device=dev)
    ctx.check(ctx.lib.vsig_psd_c64_dev(ctx.h, _ptr(xd), n, int(_stride), _ptr(wd), nperseg, hop,
                                       nfft, scale, 1 if fftshift else 0, _ptr(out), nframes),
              "spectrum")
    freqs = np.fft.fftfreq(nfft, 1 / fs)
    times = np.arange(nperseg / 2, n - nperseg / 2 + 1, hop) / float(fs)
    if _is_dev(x):
        return freqs, times, out.T
    S = out.cpu().numpy().T
    odt = _out_real_dtype(x)
    if odt == np.float64:
        S = S.astype(np.float64)
    return freqs, times, S


# ---------------------------------------------------------------------------
# filter — np.convolve(x, taps, 'full')[:len(x)][::decim]
# ---------------------------------------------------------------------------
class FirFilter:
    """Causal FIR + decimation on the GPU: ``y = np.convolve(x, taps)[:len(x)][::decim]``
    (overlap-save; the filter spectrum is computed once at construction)."""

    def __init__(self, taps, decim: int = 1, device: int | None = None):
        taps = np.ascontiguousarray(np.asarray(taps).ravel(), dtype=np.complex64)
        if taps.size == 0:
            raise ValueError("v cannot be empty")
        if int(decim) < 1:
            raise ValueError("decim must be >= 1")
        self.ctx = _lib.get_context(device)
        self.ntaps, self.decim = int(taps.size), int(decim)
        h = C.c_void_p()
        self.ctx.check(self.ctx.lib.vsig_fir_create(self.ctx.h, taps.ctypes.data_as(C.c_void_p),
                                                    self.ntaps, self.decim, C.byref(h)),
                       "vsig_fir_create")
        self.h = h

    def out_len(self, n: int) -> int:
        return (n + self.decim - 1) // self.decim

    def __call__(self, x: torch.Tensor, out: torch.Tensor | None = None,
                 nhist: int = 0, freq_shift: float = 0.0, sample_rate: float = 1.0,
                 i0: int = 0) -> torch.Tensor:
        """x: 1-D complex64 CUDA tensor -> complex64 CUDA tensor (async).
        The first nhist samples of x are history (a left halo): only the
        remaining samples produce outputs.  freq_shift != 0 filters
        apply_frequency_shift(x, freq_shift, sample_rate) instead (the NCO
        mixer fused into the filter's loads; x[0] is global sample i0)."""
        self.ctx.bind_stream()
        _check_dev(x, 1, torch.complex64, "filter input", self.ctx.device)
        n = int(x.shape[0]) - int(nhist)
        if n < 1 or nhist < 0:
            raise ValueError("filter: need len(x) > nhist >= 0")
        ny = self.out_len(n)
        if out is None:
            out = torch.empty(ny, dtype=torch.complex64, device=x.device)
        _check_dev(out, ny, torch.complex64, "filter output", self.ctx.device)
        if freq_shift and self.block != 1024:
            # long filters (M > 1024): the standalone mixer first, same phase origin
            xm = torch.empty_like(x)
            w = (2j * np.pi * freq_shift).imag
            self.ctx.check(self.ctx.lib.vsig_mix_c64_dev(self.ctx.h, _ptr(x), int(x.shape[0]),
                                                         float(w), float(sample_rate), int(i0),
                                                         _ptr(xm)), "mix")
            x, freq_shift = xm, 0.0
        if freq_shift:
            self.ctx.check(self.ctx.lib.vsig_fir_exec_mix_dev(
                self.h, _ptr(x), int(nhist), n, _ptr(out), ny, float(freq_shift),
                float(sample_rate), int(i0)), "filter (mixed)")
        else:
            self.ctx.check(self.ctx.lib.vsig_fir_exec_hist_dev(self.h, _ptr(x), int(nhist), n,
                                                               _ptr(out), ny), "filter")
        return out

    @property
    def block(self) -> int:
        """Overlap-save block size the library chose for these taps."""
        return int(self.ctx.lib.vsig_fir_block(self.h))

    def __del__(self):
        try:
            if self.h:
                self.ctx.lib.vsig_fir_free(self.h)
                self.h = None
        except Exception:
            pass


_fir_cache: "OrderedDict[tuple, FirFilter]" = OrderedDict()


def _cached_fir(taps_c64: np.ndarray, decim: int, device: int) -> FirFilter:
    key = (taps_c64.tobytes(), decim, device)
    f = _fir_cache.get(key)
    if f is None:
        f = FirFilter(taps_c64, decim, device)
        _fir_cache[key] = f
        if len(_fir_cache) > 16:
            _fir_cache.popitem(last=False)
    else:
        _fir_cache.move_to_end(key)
    return f


def fir_filter(x, taps, decim: int = 1, freq_shift: float = 0.0, sample_rate: float = 1.0):
    """Causal FIR then stride decimation: ``np.convolve(x, taps, 'full')[:len(x)][::decim]``
    (the reference's idioms, utils.py:802,816 and utils.py:194).  With
    ``freq_shift`` the input is first mixed as ``apply_frequency_shift(x,
    freq_shift, sample_rate)`` (utils.py:120-127) inside the same kernel."""
    if freq_shift and float(sample_rate) == 0.0:
        raise ZeroDivisionError("float division by zero")
    taps_np = np.asarray(taps)
    if taps_np.size == 0:
        raise ValueError("v cannot be empty")
    n = int(x.shape[0]) if _is_dev(x) else np.asarray(x).shape[0]
    if n == 0:
        raise ValueError("a cannot be empty")
    ctx = _lib.get_context()
    f = _cached_fir(np.ascontiguousarray(taps_np.ravel(), dtype=np.complex64), int(decim), ctx.device)
    xd = _device_c64(x, ctx)
    y = f(xd, freq_shift=freq_shift, sample_rate=sample_rate)
    if _is_dev(x):
        return y
    xa = np.asarray(x)
    odt = np.result_type(xa.dtype, taps_np.dtype)
    yh = y.cpu().numpy()
    if not np.issubdtype(odt, np.complexfloating):
        yh = yh.real
    return yh.astype(odt, copy=False)


filter = fir_filter  # noqa: A001  (north-star name)


# ---------------------------------------------------------------------------
# correlation
# ---------------------------------------------------------------------------
def _lags(mode, l1, l2):
    """utils.py:1288-1293 (incl. the 'same'-mode length quirk)."""
    if mode == "full":
        return np.arange(-l1 + 1, l2)
    if mode == "same":
        return np.arange(-l1 // 2, l1 // 2 + l1 % 2)
    return np.arange(l2 - l1 + 1)


def _corr_len(mode, na, nv):
    if mode == "full":
        return na + nv - 1
    if mode == "valid":
        return max(na, nv) - min(na, nv) + 1
    return max(na, nv)


def _check_mode(mode):
    if mode not in _lib.MODES:
        raise ValueError(f"mode must be one of 'full', 'valid', 'same' (got {mode!r})")


def _is_c128(x) -> bool:
    """Does the reference's complex128 upcast (utils.py:1279-1282) change x's
    values?  complex64 / float32 data upcast exactly (the complex64 path is
    then numpy's arithmetic on the same values); wider dtypes keep 128 bits."""
    if _is_dev(x):
        return x.dtype in (torch.complex128, torch.float64, torch.int64, torch.int32)
    dt = np.asarray(x).dtype
    return not (dt == np.complex64 or dt == np.float32 or dt == np.float16
                or dt == np.int8 or dt == np.uint8 or dt == np.int16 or dt == np.uint16)


def _device_c128(x, ctx):
    if _is_dev(x):
        t = x if x.is_cuda else x.to(f"cuda:{ctx.device}")
        return t.to(torch.complex128).contiguous()
    a = np.ascontiguousarray(np.asarray(x), dtype=np.complex128)
    if a.ndim != 1:
        raise ValueError("vector_amd works on 1-D signals")
    return torch.from_numpy(a).to(f"cuda:{ctx.device}")


def _correlate_dev(a, v, mode, want_array, ctx, out128=False):
    """np.correlate(a, v, mode) on the GPU; returns (c tensor or None, peak
    buffer, nout).  complex128 operands (or any input whose complex128 upcast
    is not exact) go to the library as complex128: the FFT pass runs in
    complex64, the argmax refine (refine.hip) in the operands' precision.
    out128: c is returned as complex128 with the refined outputs patched in."""
    in128 = _is_c128(a) or _is_c128(v)
    conv = _device_c128 if in128 else _device_c64
    ad, vd = conv(a, ctx), conv(v, ctx)
    ctx.sync_blas_threads()
    na, nv = int(ad.shape[0]), int(vd.shape[0])
    if na == 0:
        raise ValueError("a cannot be empty")
    if nv == 0:
        raise ValueError("v cannot be empty")
    nout = _corr_len(mode, na, nv)
    odt = torch.complex128 if out128 else torch.complex64
    c = torch.empty(nout, dtype=odt, device=ad.device) if want_array else None
    pk = _peak_buffer(ctx)
    ctx.check(ctx.lib.vsig_correlate_dev(ctx.h, _lib.DTYPES["c128" if in128 else "c64"], _ptr(ad),
                                         na, _ptr(vd), nv, _lib.MODES[mode],
                                         _lib.DTYPES["c128" if out128 else "c64"],
                                         _ptr(c) if c is not None else None, _ptr(pk)),
              "correlate")
    return c, pk, nout, (ad, vd, in128)


def refine_status(ctx=None):
    """(status, candidates) of the last correlation's argmax refine:
    0 refined, 1 skipped (more candidate outputs than a 'refine_cap' option
    set > 0; the default is no limit), 2 no refine pass ran, 3 the refine's
    watchdog fired since the last call (vsig.h vsig_refine_status; reported
    once, the refine's counters are cleared by the call)."""
    ctx = ctx or _lib.get_context()
    st, nc = C.c_int32(), C.c_int64()
    ctx.check(ctx.lib.vsig_refine_status(ctx.h, C.byref(st), C.byref(nc)), "refine_status")
    return int(st.value), int(nc.value)


def check_refine(ctx=None):
    """The exact-argmax contract after a correlation: status 3 (the refine's
    watchdog fired: a device fault) raises RefineFault; status 1 (an opt-in
    'refine_cap' exceeded) warns -- that limit is the caller's own choice.
    Device-tensor callers (Correlator, cross_correlate_signals on CUDA
    tensors) run asynchronously and call this themselves when they read the
    result (StreamChain.global_peak does)."""
    ctx = ctx or _lib.get_context()
    st, nc = refine_status(ctx)
    if st == 3:
        raise _lib.RefineFault("correlation argmax refine: watchdog fired (device fault); the "
                               "peak record is invalid (vsig_refine_status 3)")
    if st == 1:
        warnings.warn(f"correlation argmax left at fp32 accuracy: the {nc} candidate items within "
                      f"the refine band exceed the 'refine_cap' option", RuntimeWarning, stacklevel=3)


def cross_correlate_signals(signal1, signal2, mode="full"):
    """utils.py:1258-1295: ``np.correlate(signal2, signal1, mode)`` and the lag
    axis.  numpy inputs -> complex128 numpy: the FFT pass runs in complex64, the
    outputs within the refine band of the peak -- however many (a tone puts
    every full-overlap output there) -- are recomputed in numpy's own
    operation order, so find_correlation_peak over the result gives numpy's
    argmax and |c| to the bit; elsewhere complex64 accuracy.  A 'refine_cap'
    option > 0 (an explicit opt-in; default none) leaves a larger band at
    fp32 accuracy with a RuntimeWarning (refine_status)."""
    _check_mode(mode)
    ctx = _lib.get_context()
    dev = _is_dev(signal1) or _is_dev(signal2)
    out128 = (not dev) or _is_c128(signal1) or _is_c128(signal2)
    c, _, _, _ = _correlate_dev(signal2, signal1, mode, True, ctx, out128=out128)
    l1 = int(signal1.shape[0]) if _is_dev(signal1) else len(signal1)
    l2 = int(signal2.shape[0]) if _is_dev(signal2) else len(signal2)
    lags = _lags(mode, l1, l2)
    if dev:
        return c, lags
    out = c.cpu().numpy()
    check_refine(ctx)
    return out, lags


correlate = cross_correlate_signals


def _stats_operand(a, ctx):
    """a as a contiguous CUDA tensor and its dtype code."""
    if _is_dev(a):
        t = a.contiguous()
        code = {torch.complex128: "c128", torch.complex64: "c64", torch.float64: "f64",
                torch.float32: "f32"}.get(t.dtype)
        if code is None:
            t, code = t.to(torch.float64), "f64"
    else:
        arr = np.asarray(a)
        if arr.dtype == np.complex128:
            code = "c128"
        elif arr.dtype == np.complex64:
            code = "c64"
        elif arr.dtype == np.float32:
            code = "f32"
        elif np.iscomplexobj(arr):
            arr, code = arr.astype(np.complex128), "c128"
        else:
            arr, code = arr.astype(np.float64), "f64"
        t = torch.from_numpy(np.ascontiguousarray(arr.ravel())).to(f"cuda:{ctx.device}")
    return t, code


def peak_stats(a):
    """(argmax of |a| (first), max |a|, sum |a|, sum |a|^2, n) in double
    precision on the GPU, for numpy or CUDA arrays of complex/real dtype."""
    ctx = _lib.get_context()
    t, code = _stats_operand(a, ctx)
    n = int(t.numel())
    if n == 0:
        raise ValueError("attempt to get argmax of an empty sequence")
    pk = _peak_buffer(ctx)
    ctx.check(ctx.lib.vsig_peak_dev(ctx.h, _lib.DTYPES[code], _ptr(t), n, _ptr(pk)), "peak")
    mx, idx, s1, s2 = _read_peak(pk)
    return idx, mx, s1, s2, n


def find_correlation_peak(correlation, lags, threshold_ratio=0.5):
    """utils.py:1298-1342 — (lags[argmax |c|], max |c|, confidence).
    complex128 / float64 arrays (cross_correlate_signals' output): mean and std
    of |c| exactly as numpy forms them (its pairwise sums, two passes); other
    dtypes: from double sums of |c| (single pass)."""
    ctx = _lib.get_context()
    t, code = _stats_operand(correlation, ctx)
    n = int(t.numel())
    if n == 0:
        raise ValueError("attempt to get argmax of an empty sequence")
    pk = _peak_buffer(ctx)
    ctx.check(ctx.lib.vsig_peak_dev(ctx.h, _lib.DTYPES[code], _ptr(t), n, _ptr(pk)), "peak")
    peak, idx, s1, s2 = _read_peak(pk)
    if code in ("c128", "f64"):
        mean, std = _abs_stats(t, code, ctx)
    else:
        mean, std, _ = _fused_stats(peak, s1, s2, n)
    return lags[idx], np.float64(peak), _confidence_np(peak, mean, std, threshold_ratio)


def correlate_peak(signal1, signal2, mode="full", threshold_ratio=0.5):
    """``find_correlation_peak(*cross_correlate_signals(signal1, signal2, mode))``
    fused: the correlation is reduced inside the kernel and never stored."""
    _check_mode(mode)
    ctx = _lib.get_context()
    _, pk, nout, (ad, vd, in128) = _correlate_dev(signal2, signal1, mode, False, ctx)
    peak, idx, s1, s2 = _read_peak(pk)
    check_refine(ctx)
    mean, std, resolved = _fused_stats(peak, s1, s2, nout)
    if not resolved:
        # a (nearly) flat |c|: numpy's std is decided by rounding; every
        # output's |c| in numpy's order, then numpy's two-pass statistics
        st = torch.empty(2, dtype=torch.float64, device=ad.device)
        ctx.check(ctx.lib.vsig_correlate_stats_dev(
            ctx.h, _lib.DTYPES["c128" if in128 else "c64"], _ptr(ad), int(ad.shape[0]), _ptr(vd),
            int(vd.shape[0]), _lib.MODES[mode], _ptr(st)), "correlate stats")
        mean, std = (np.float64(x) for x in st.cpu().tolist())
    conf = _confidence_np(peak, mean, std, threshold_ratio)
    l1 = int(signal1.shape[0]) if _is_dev(signal1) else len(signal1)
    l2 = int(signal2.shape[0]) if _is_dev(signal2) else len(signal2)
    if mode == "full":
        lag = np.int64(idx - (l1 - 1))
    elif mode == "valid":
        if idx >= l2 - l1 + 1:          # lag axis np.arange(l2 - l1 + 1) (utils.py:1291)
            raise IndexError(f"index {idx} is out of bounds for axis 0 with size "
                             f"{max(0, l2 - l1 + 1)}")
        lag = np.int64(idx)
    else:
        lag = _lags(mode, l1, l2)[idx]      # raises IndexError like the reference
    return lag, np.float64(peak), conf


class Correlator:
    """Streaming sync detector: a fixed template (any length; > 8192 samples
    runs as one pass per 8192-sample chunk), correlated against long
    device-resident streams with the |c| argmax fused in the kernel and
    refined (refine.hip) -- all asynchronous on the current stream."""

    def __init__(self, template, device: int | None = None):
        t = np.ascontiguousarray(np.asarray(template).ravel(), dtype=np.complex64)
        if t.size == 0:
            raise ValueError("v cannot be empty")
        self.ctx = _lib.get_context(device)
        self.L = int(t.size)
        self.h = None
        h = C.c_void_p()
        self.ctx.check(self.ctx.lib.vsig_xcorr_create(self.ctx.h, t.ctypes.data_as(C.c_void_p),
                                                      self.L, C.byref(h)), "vsig_xcorr_create")
        self.h = h

    def __call__(self, s: torch.Tensor, mode="valid", out: torch.Tensor | None = None,
                 peak: torch.Tensor | None = None):
        """Enqueue; returns (c or None, peak buffer (device vsig_peak_t)).  The
        refine matches numpy's current OpenBLAS thread count, as the numpy
        front end does (Context.sync_blas_threads: one C call)."""
        self.ctx.bind_stream()
        self.ctx.sync_blas_threads()
        _check_dev(s, 1, torch.complex64, "correlator stream", self.ctx.device)
        if mode not in ("valid", "full"):
            raise ValueError("Correlator supports mode 'valid' and 'full'")
        ns = int(s.shape[0])
        nout = ns - self.L + 1 if mode == "valid" else ns + self.L - 1
        if nout < 1:
            raise ValueError("stream shorter than the template")
        if out is not None:
            _check_dev(out, nout, torch.complex64, "correlator output", self.ctx.device)
        if peak is None:
            peak = _peak_buffer(self.ctx)
        _check_dev(peak, 4, torch.float64, "peak record", self.ctx.device)
        self.ctx.check(self.ctx.lib.vsig_xcorr_exec_dev(
            self.h, _ptr(s), ns, _lib.MODES[mode],
            _ptr(out) if out is not None else None, _ptr(peak)), "xcorr")
        return out, peak

    def __del__(self):
        try:
            if self.h:
                self.ctx.lib.vsig_xcorr_free(self.h)
                self.h = None
        except Exception:
            pass


def find_packet_location_in_vector(vector, packet_signal, reference_segment,
                                   search_window=None, correlation_threshold=0.5):
    """utils.py:1372-1434 with both correlations reduced on the GPU."""
    if search_window is None:
        s0, s1 = 0, len(vector)
    else:
        s0, s1 = search_window
        s0, s1 = max(0, s0), min(len(vector), s1)
    vlag, _, vconf = correlate_peak(reference_segment, vector[s0:s1], "full", correlation_threshold)
    plag, _, pconf = correlate_peak(reference_segment, packet_signal, "full", correlation_threshold)
    return s0 + vlag - plag, 0, min(vconf, pconf)
