"""Detection / display helpers of the reference on the GPU (SURVEY.md §8(a)
rows a3, a7, a8):

  normalize_spectrogram   utils.py:356-404
  find_packet_start       utils.py:784-809
  detect_packet_bounds    utils.py:811-825

The data-parallel work — |S| order statistics, the dB transform, the |x|^2
prefix scan and boxcar smoothing, the threshold scan, the magnitude
correlation — runs in libvsig.so (analysis.hip, psd.hip, xcorr.hip, reduce.hip).  What is left on
the host is O(1) scalar arithmetic, written so that numpy's own rules
(np.percentile 'linear' in the array's dtype, np.median, NEP 50 promotion)
give the same numbers the reference computes.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from . import _lib
from .dsp import _correlate_dev, _is_dev, _ptr

__all__ = ["normalize_spectrogram", "find_packet_start", "detect_packet_bounds",
           "order_statistics", "threshold_stats", "boxcar_energy"]

_TORCH_CODE = {torch.complex128: "c128", torch.complex64: "c64", torch.float64: "f64",
               torch.float32: "f32"}
_NP_CODE = {np.dtype(np.complex128): "c128", np.dtype(np.complex64): "c64",
            np.dtype(np.float64): "f64", np.dtype(np.float32): "f32"}


def _to_device(x, ctx, real_only=False):
    """(flat contiguous CUDA tensor, dtype code) keeping numpy's dtype where the
    kernels support it (other dtypes go to float64 / complex128 as numpy's
    promotion would for these expressions)."""
    if _is_dev(x):
        t = x
        if not t.is_cuda:
            t = t.to(f"cuda:{ctx.device}")
        code = _TORCH_CODE.get(t.dtype)
        if code is None:
            t = t.to(torch.complex128 if t.is_complex() else torch.float64)
            code = _TORCH_CODE[t.dtype]
        t = t.contiguous().reshape(-1)
    else:
        a = np.asarray(x)
        code = _NP_CODE.get(a.dtype)
        if code is None:
            a = a.astype(np.complex128 if np.iscomplexobj(a) else np.float64)
            code = _NP_CODE[a.dtype]
        t = torch.from_numpy(np.ascontiguousarray(a).reshape(-1)).to(f"cuda:{ctx.device}")
    if real_only and code in ("c64", "c128"):
        raise ValueError("expected a real array")
    return t, code


def order_statistics(a, ranks):
    """k-th smallest |a| (0-based) for up to 4 ranks — MSB-first radix select
    on the GPU (real float32 / float64 data)."""
    ctx = _lib.get_context()
    t, code = _to_device(a, ctx, real_only=True)
    return _order_stats_dev(ctx, t, code, ranks)


def _order_stats_dev(ctx, t, code, ranks):
    ranks = [int(r) for r in ranks]
    out = []
    for i in range(0, len(ranks), 4):
        rk = ranks[i:i + 4]
        rarr = (C.c_int64 * len(rk))(*rk)
        vals = (C.c_double * len(rk))()
        ctx.check(ctx.lib.vsig_select_dev(ctx.h, _lib.DTYPES[code], _ptr(t), int(t.numel()), rarr,
                                          len(rk), vals), "select")
        out.extend(vals[:len(rk)])
    return out


def threshold_stats(a, thr):
    """(count, first, last, max) of |a| >= thr over a real array (first = n,
    last = -1 when nothing passes)."""
    ctx = _lib.get_context()
    t, code = _to_device(a, ctx, real_only=True)
    return _thresh_dev(ctx, t, code, thr)


def _thresh_dev(ctx, t, code, thr):
    cnt, first, last = C.c_int64(), C.c_int64(), C.c_int64()
    mx = C.c_double()
    ctx.check(ctx.lib.vsig_threshold_dev(ctx.h, _lib.DTYPES[code], _ptr(t), int(t.numel()),
                                         float(thr), C.byref(cnt), C.byref(first), C.byref(last),
                                         C.byref(mx)), "threshold")
    return cnt.value, first.value, last.value, mx.value


def boxcar_energy(signal, w):
    """np.convolve(np.abs(signal) ** 2, np.ones(w) / w, 'same') as a float64
    CUDA tensor (length max(n, w))."""
    ctx = _lib.get_context()
    t, code = _to_device(signal, ctx)
    return _boxcar_dev(ctx, t, code, w)


def _boxcar_dev(ctx, t, code, w):
    n = int(t.numel())
    if n == 0:
        raise ValueError("v cannot be empty")
    sm = torch.empty(max(n, int(w)), dtype=torch.float64, device=t.device)
    ctx.check(ctx.lib.vsig_boxcar_energy_dev(ctx.h, _lib.DTYPES[code], _ptr(t), n, int(w), _ptr(sm)),
              "boxcar")
    return sm


# ---------------------------------------------------------------------------
# numpy's order-statistic reductions restated over GPU order statistics
# ---------------------------------------------------------------------------
def _percentile(n, pct, dt, fetch):
    """np.percentile(arr, pct) (method 'linear') for an array of n elements
    of dtype dt, given fetch(ranks) -> k-th smallest values.  Mirrors numpy's
    _quantile / _get_indexes / _get_gamma / _lerp including the dtype the
    arithmetic runs in (float32 arrays interpolate in float32)."""
    dt = np.dtype(dt)
    q = np.asanyarray(np.true_divide(pct, dt.type(100)))
    if np.any(q < 0) or np.any(q > 1):
        raise ValueError("Percentiles must be in the range [0, 100]")
    virtual = np.asanyarray((n - 1) * q)
    prev = np.asanyarray(np.floor(virtual))
    nxt = prev + 1
    if virtual >= n - 1:
        prev, nxt = np.asanyarray(-1), np.asanyarray(-1)
    if virtual < 0:
        prev, nxt = np.asanyarray(0), np.asanyarray(0)
    if np.isnan(virtual):
        prev, nxt = np.asanyarray(-1), np.asanyarray(-1)
    pi, ni = int(prev) % n, int(nxt) % n
    vals = fetch(sorted({pi, ni}))
    a = np.asarray(vals[pi], dtype=dt)
    b = np.asarray(vals[ni], dtype=dt)
    gamma = np.asanyarray(virtual - prev.astype(np.intp), dtype=virtual.dtype)
    diff = np.subtract(b, a)
    res = np.asanyarray(np.add(a, diff * gamma))
    np.subtract(b, diff * (1 - gamma), out=res, where=gamma >= 0.5, casting="unsafe",
                dtype=res.dtype)
    return res[()]


def _median(n, dt, fetch):
    """np.median of n elements of dtype dt from order statistics."""
    if n == 0:
        return np.dtype(dt).type(np.nan)
    k = n // 2
    if n % 2:
        return np.dtype(dt).type(fetch([k])[k])
    v = fetch([k - 1, k])
    return np.mean(np.array([v[k - 1], v[k]], dtype=dt))


# ---------------------------------------------------------------------------
# normalize_spectrogram — utils.py:356-404
# ---------------------------------------------------------------------------
def normalize_spectrogram(Sxx, low_percentile=10.0, high_percentile=95.0, max_dynamic_range=25):
    """utils.py:356-404: (Sxx_db, vmin, vmax) with Sxx_db = 10 log10(|S| + floor),
    floor = max(5th percentile of the positive |S|, 1e-12), vmin / vmax the
    10th / 95th percentiles of Sxx_db, then the dynamic-range clamps.

    The percentiles come from radix-select order statistics of |S| on the GPU:
    10 log10(. + floor) is non-decreasing, so the k-th smallest dB value is
    the transform of the k-th smallest |S|.  numpy in -> numpy out; a CUDA
    tensor in -> Sxx_db stays on the device."""
    dev_in = _is_dev(Sxx)
    size = int(Sxx.numel()) if dev_in else int(np.size(Sxx))
    if size == 0:
        return np.array([]), 0, 0
    ctx = _lib.get_context()
    shape = tuple(Sxx.shape)
    # transposed views (spectrum() returns (nfft, frames) over frame-major
    # memory) are reduced in their storage order and returned in the same view
    src = Sxx
    transposed = False
    if dev_in and Sxx.dim() == 2 and not Sxx.is_contiguous() and Sxx.t().is_contiguous():
        src, transposed = Sxx.t(), True
    t, code = _to_device(src, ctx, real_only=True)
    dt = np.float32 if code == "f32" else np.float64
    n = int(t.numel())
    cache = {}

    def fetch(ranks, base=0):
        need = [r for r in ranks if r + base not in cache]
        if need:
            got = _order_stats_dev(ctx, t, code, [r + base for r in need])
            cache.update({r + base: v for r, v in zip(need, got)})
        return {r: cache[r + base] for r in ranks}

    # |S| > 0 count: |S| >= the smallest subnormal of the dtype
    tiny = float(np.finfo(dt).smallest_subnormal)
    npos, _, _, _ = _thresh_dev(ctx, t, code, tiny)
    if npos > 0:
        nzero = n - npos
        noise_floor = _percentile(npos, 5, dt, lambda rk: fetch(rk, nzero))
    else:
        noise_floor = 1e-12
    noise_floor = max(noise_floor, 1e-12)
    # numpy's promotion of |S| + noise_floor (NEP 50: a Python float is weak)
    db_dt = np.result_type(np.empty(0, dt), noise_floor)
    floor_v = float(np.asarray(noise_floor, dtype=db_dt))
    out_t = torch.float32 if db_dt == np.float32 else torch.float64
    if db_dt == np.float64 and code == "f32":
        t = t.to(torch.float64)
        code = "f64"
    db = torch.empty(n, dtype=out_t, device=t.device)
    ctx.check(ctx.lib.vsig_db_dev(ctx.h, _lib.DTYPES[code], _ptr(t), n, floor_v, _ptr(db)), "db")

    def db_of(v):
        return 10 * np.log10(np.asarray(v, dtype=db_dt) + np.asarray(floor_v, dtype=db_dt))

    def fetch_db(ranks):
        return {r: db_of(v) for r, v in fetch(ranks).items()}

    try:
        vmin = _percentile(n, low_percentile, db_dt, fetch_db)
        vmax = _percentile(n, high_percentile, db_dt, fetch_db)
    except Exception:
        vmin, vmax = db_of(fetch([0])[0])[()], db_of(fetch([n - 1])[n - 1])[()]
    if np.isnan(vmin) or np.isnan(vmax) or vmax <= vmin:
        vmin, vmax = db_of(fetch([0])[0])[()], db_of(fetch([n - 1])[n - 1])[()]
        if vmax <= vmin:
            vmax = vmin + max_dynamic_range
    actual_range = vmax - vmin
    if actual_range > max_dynamic_range:
        vmin = vmax - max_dynamic_range
    elif actual_range < 20:
        mid_point = (vmax + vmin) / 2
        vmin = mid_point - 10
        vmax = mid_point + 10
    vmin = max(vmin, -120)
    if actual_range != vmax - vmin:
        print(f"📊 Dynamic range adjusted: {actual_range:.1f}dB → {vmax - vmin:.1f}dB "
              "(optimized for resolution)")
    if transposed:
        db = db.reshape(tuple(src.shape)).t()
    else:
        db = db.reshape(shape)
    if dev_in:
        return db, vmin, vmax
    return db.cpu().numpy(), vmin, vmax


# ---------------------------------------------------------------------------
# find_packet_start / detect_packet_bounds — utils.py:784-825
# ---------------------------------------------------------------------------
def _threshold_first_last(ctx, sm, m, threshold_ratio):
    """noise = median(sm[:m]), thr = noise + r (max - noise), first / last
    index of sm >= thr (count 0 -> None)."""
    head = sm[:m]
    cache = {}

    def fetch(ranks):
        need = [r for r in ranks if r not in cache]
        if need:
            cache.update(zip(need, _order_stats_dev(ctx, head, "f64", need)))
        return {r: cache[r] for r in ranks}

    noise = _median(m, np.float64, fetch)
    _, _, _, max_en = _thresh_dev(ctx, sm, "f64", np.inf)
    threshold = noise + threshold_ratio * (np.float64(max_en) - noise)
    if np.isnan(threshold):
        return None
    cnt, first, last, _ = _thresh_dev(ctx, sm, "f64", float(threshold))
    if cnt == 0:
        return None
    return first, last


def find_packet_start(signal, template=None, threshold_ratio=0.2, window_size=None):
    """utils.py:784-809.  Template branch: argmax of
    np.correlate(|signal|, |template|, 'valid') (overlap-save correlator on the
    magnitudes, argmax fused); energy branch: boxcar-smoothed |x|^2 (prefix
    scan), median of the first 10 % (radix select), first index above
    noise + r (max - noise)."""
    ctx = _lib.get_context()
    if template is not None:
        s, scode = _to_device(signal, ctx)
        tm, tcode = _to_device(template, ctx)
        if s.numel() == 0 or tm.numel() == 0:
            raise ValueError("v cannot be empty" if tm.numel() == 0 else "a cannot be empty")
        # np.abs keeps the input's precision: complex64 / float32 magnitudes are
        # float32 (exact in complex64), wider ones float64 (complex128 operands
        # of the correlation, so the argmax refine sees numpy's values)
        wide = scode in ("c128", "f64") or tcode in ("c128", "f64")
        odt = torch.complex128 if wide else torch.complex64
        absfn = ctx.lib.vsig_abs_c128_dev if wide else ctx.lib.vsig_abs_c64_dev
        sa = torch.empty(int(s.numel()), dtype=odt, device=s.device)
        ta = torch.empty(int(tm.numel()), dtype=odt, device=s.device)
        ctx.check(absfn(ctx.h, _lib.DTYPES[scode], _ptr(s), int(s.numel()), _ptr(sa)), "abs")
        ctx.check(absfn(ctx.h, _lib.DTYPES[tcode], _ptr(tm), int(tm.numel()), _ptr(ta)), "abs")
        _, pk, _, _ = _correlate_dev(sa, ta, "valid", False, ctx)
        return int(pk.cpu().view(torch.int64)[1].item())
    t, code = _to_device(signal, ctx)
    n = int(t.numel())
    if window_size is None:
        window_size = max(1, int(0.02 * n))
    w = max(1, window_size)
    sm = _boxcar_dev(ctx, t, code, w)
    r = _threshold_first_last(ctx, sm, int(sm.numel()) // 10, threshold_ratio)
    return int(r[0]) if r is not None else 0


def detect_packet_bounds(signal, sample_rate, threshold_ratio=0.2):
    """utils.py:811-825: (start, end) of the smoothed-energy burst (1 us
    boxcar), (0, len(signal)) when nothing passes the threshold."""
    ctx = _lib.get_context()
    t, code = _to_device(signal, ctx)
    n = int(t.numel())
    w = max(1, int(sample_rate // 1_000_000))
    sm = _boxcar_dev(ctx, t, code, w)
    r = _threshold_first_last(ctx, sm, max(1, int(sm.numel()) // 10), threshold_ratio)
    if r is None:
        return 0, n
    return np.int64(r[0]), np.int64(r[1])
