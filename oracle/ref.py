"""CPU oracle for the vector-signal DSP hot path — TEST INFRASTRUCTURE ONLY.

This module is the parity checker, never the product.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
it.  The product (``vector_amd``) must never import or call anything here; it
fails loudly when its HIP library is missing instead of falling back to a CPU
path.

It restates, in plain NumPy/SciPy, the semantics of the reference's DSP
functions (ramiyako/vector ``utils.py``, snapshot 2025-07-18).  The reference's
arithmetic itself lives in third-party code that is *not* vendored under
``/root/reference``: numpy 2.2.6 (``np.correlate`` -> ``multiarray.correlate2``,
``np.convolve`` -> ``multiarray.correlate``, ``numpy/_core/numeric.py:693-869``)
and scipy 1.15.3 (``scipy.signal.spectrogram`` -> ``_spectral_helper`` ->
``_fft_helper`` -> pocketfft, ``scipy/signal/_spectral_py.py:816-2205``).
Requirements pin only lower bounds (``requirements.txt``: numpy>=1.21,
scipy>=1.7).  This oracle calls those same library routines, so its numerics are
the reference's numerics.

Pinning: every function below is checked against golden vectors produced by
importing the reference's own ``utils`` in the build container
(``tests/golden/make_golden.py`` -> ``tests/golden/*.npz``) and against the
known answers of the reference's tests (``tests/test_utils.py:24-34``,
``test_packet_transplant.py:40-68``).  ``fir_filter`` and ``pfb_channelize`` have
no reference function: they are pinned by numpy semantics
only ("parity unpinned" at the reference level).
"""
from __future__ import annotations

import numpy as np
import scipy.signal

__all__ = [
    "spectrum", "spectrogram_params", "create_spectrogram", "normalize_spectrogram",
    "cross_correlate_signals", "find_correlation_peak", "xcorr_peak",
    "find_packet_location_in_vector", "find_packet_start", "detect_packet_bounds",
    "fir_filter", "stride_decimate", "pfb_channelize", "synth_iq", "qpsk_preamble",
]


# ---------------------------------------------------------------------------
# spectrum — utils.py:281-291 (scipy.signal.spectrogram, two-sided, 'spectrum')
# ---------------------------------------------------------------------------
def spectrum(x, fs=1.0, window="hann", nperseg=256, noverlap=None, nfft=None):
    """``scipy.signal.spectrogram`` exactly as the reference calls it
    (utils.py:281-291): ``return_onesided=False, detrend=False,
    scaling='spectrum'``.  Returns ``(f, t, Sxx)``; ``Sxx`` is (nfft, nframes)."""
    return scipy.signal.spectrogram(
        x, fs=fs, window=window, nperseg=nperseg, noverlap=noverlap, nfft=nfft,
        return_onesided=False, detrend=False, scaling="spectrum")


def spectrogram_params(n, sr, max_samples=2_000_000, time_resolution_us=1,
                       adaptive_resolution=True):
    """Host-side parameter selection of ``create_spectrogram``
    (utils.py:183-276), restated without the STFT call.

    Returns a dict with factor, fs, nsig (samples after stride decimation),
    window, nperseg, noverlap, nfft, heavy.
    """
    if n == 0:
        raise ValueError("Signal is empty")
    heavy = n > 5_000_000                                     # utils.py:184
    if heavy:
        max_samples = min(max_samples, 1_000_000)             # utils.py:188
        time_resolution_us = max(time_resolution_us, 20)      # utils.py:189
    if n > max_samples:                                       # utils.py:192-195
        factor = int(np.ceil(n / max_samples))
        nsig = len(range(0, n, factor))
        fs = sr / factor
    else:
        factor = 1
        nsig = n
        fs = sr
    dur_us = nsig / fs * 1e6                                  # utils.py:203
    if adaptive_resolution:                                   # utils.py:206-234
        if dur_us <= 50:
            base_window = max(32, min(nsig // 12, 128))
            time_resolution_us = min(time_resolution_us, dur_us / 10)
            frf = 1.2
        elif dur_us <= 500:
            base_window = max(64, min(nsig // 10, 256))
            time_resolution_us = min(time_resolution_us, dur_us / 20)
            frf = 1.2
        elif dur_us <= 5000:
            base_window = max(128, min(nsig // 8, 512))
            time_resolution_us = min(time_resolution_us, 10)
            frf = 1.5
        else:
            base_window = max(256, min(nsig // 6, 1024))
            time_resolution_us = min(time_resolution_us, 20)
            frf = 1.5
            if heavy:
                base_window = min(base_window, 512)
                time_resolution_us = max(time_resolution_us, 50)
                frf = 1.2
    else:
        base_window = max(128, min(nsig // 8, 512))
        frf = 1.2
    if time_resolution_us is not None:                        # utils.py:237-252
        step = max(1, int(round(fs * time_resolution_us / 1e6)))
        step = min(step, nsig // 10)
        step = max(1, step)
        window_size = max(base_window, step * 2)
        window_size = min(window_size, nsig)
        if heavy:
            overlap = max(0, window_size - step * 2)
        else:
            overlap = max(0, window_size - step)
    else:                                                     # utils.py:253-259
        window_size = min(base_window, nsig)
        overlap = int(window_size * 0.75) if heavy else int(window_size * 0.90)
    nfft = max(256, int(2 ** np.ceil(np.log2(window_size * frf))))  # :262
    nfft = min(nfft, 1024) if heavy else max(nfft, 512)       # utils.py:265-268
    window = "hann" if heavy else "blackmanharris"            # utils.py:273-276
    return dict(factor=factor, fs=fs, nsig=nsig, window=window,
                nperseg=window_size, noverlap=overlap, nfft=nfft, heavy=heavy)


def create_spectrogram(sig, sr, center_freq=0, max_samples=2_000_000,
                       time_resolution_us=1, adaptive_resolution=True):
    """Restatement of ``create_spectrogram`` (utils.py:161-353): parameter
    logic, stride decimation, STFT, the two fallback branches and fftshift."""
    sig = np.asarray(sig)
    p = spectrogram_params(len(sig), sr, max_samples, time_resolution_us,
                           adaptive_resolution)
    factor, fs = p["factor"], p["fs"]
    if factor > 1:
        sig = sig[::factor]
    try:                                                      # utils.py:279-313
        freqs, times, Sxx = spectrum(sig, fs, p["window"], p["nperseg"],
                                     p["noverlap"], p["nfft"])
    except Exception:
        ws = min(256, len(sig))
        freqs, times, Sxx = spectrum(sig, fs, "hann", ws, ws // 2, 512)
    if np.max(Sxx) == 0:                                      # utils.py:316-347
        ws = min(64, len(sig) // 4)
        try:
            freqs, times, Sxx = spectrum(sig, fs, "hann", ws, ws // 4, max(128, ws))
        except Exception:
            freqs, times, Sxx = spectrum(sig, fs, "boxcar", 32, 16, 64)
    freqs = np.fft.fftshift(freqs) * factor + center_freq    # utils.py:350
    Sxx = np.fft.fftshift(Sxx, axes=0)                        # utils.py:351
    return freqs, times, Sxx


def normalize_spectrogram(Sxx, low_percentile=10.0, high_percentile=95.0,
                          max_dynamic_range=25):
    """Restatement of ``normalize_spectrogram`` (utils.py:356-404), minus prints."""
    if Sxx.size == 0:
        return np.array([]), 0, 0
    a = np.abs(Sxx)
    nf = np.percentile(a[a > 0], 5) if np.any(a > 0) else 1e-12
    nf = max(nf, 1e-12)
    db = 10 * np.log10(a + nf)
    try:
        vmin = np.percentile(db, low_percentile)
        vmax = np.percentile(db, high_percentile)
    except Exception:
        vmin, vmax = np.min(db), np.max(db)
    if np.isnan(vmin) or np.isnan(vmax) or vmax <= vmin:
        vmin, vmax = np.min(db), np.max(db)
        if vmax <= vmin:
            vmax = vmin + max_dynamic_range
    rng = vmax - vmin
    if rng > max_dynamic_range:
        vmin = vmax - max_dynamic_range
    elif rng < 20:
        mid = (vmax + vmin) / 2
        vmin, vmax = mid - 10, mid + 10
    vmin = max(vmin, -120)
    return db, vmin, vmax


# ---------------------------------------------------------------------------
# correlation — utils.py:1258-1342, 1372-1434, 793-795
# ---------------------------------------------------------------------------
def cross_correlate_signals(signal1, signal2, mode="full"):
    """utils.py:1258-1295: upcast to complex128, ``np.correlate(signal2,
    signal1, mode)`` (conjugates signal1), plus the lag axis (incl. the
    'same'-mode lag-length quirk)."""
    s1 = np.asarray(signal1).astype(np.complex128)
    s2 = np.asarray(signal2).astype(np.complex128)
    c = np.correlate(s2, s1, mode=mode)
    if mode == "full":
        lags = np.arange(-len(s1) + 1, len(s2))
    elif mode == "same":
        lags = np.arange(-len(s1) // 2, len(s1) // 2 + len(s1) % 2)
    else:
        lags = np.arange(len(s2) - len(s1) + 1)
    return c, lags


def find_correlation_peak(correlation, lags, threshold_ratio=0.5):
    """utils.py:1298-1342: first-max argmax of |c|, z-score confidence / 10
    clipped to [0, 1] (population std)."""
    a = np.abs(correlation)
    i = int(np.argmax(a))
    peak = a[i]
    m, s = np.mean(a), np.std(a)
    conf = float(np.clip((peak - m) / s / 10.0, 0.0, 1.0)) if s > 0 else 0.0
    if peak < threshold_ratio * np.max(a):
        conf = 0.0
    return lags[i], peak, conf


def _np_pairwise(a, off, n):
    """numpy's pairwise_sum (numpy 2.2 _core/src/umath/loops_utils.h.src) over
    a[off:off+n] in float64: < 8 elements summed from -0.0; <= 128 with 8
    accumulators, their fixed tree, then the tail; else split at n / 2 rounded
    down to a multiple of 8."""
    if n < 8:
        r = -0.0
        for i in range(n):
            r += a[off + i]
        return r
    if n <= 128:
        r = [a[off + j] for j in range(8)]
        i = 8
        while i < n - (n % 8):
            for j in range(8):
                r[j] += a[off + i + j]
            i += 8
        res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]))
        while i < n:
            res += a[off + i]
            i += 1
        return res
    h = n // 2
    h -= h % 8
    return _np_pairwise(a, off, h) + _np_pairwise(a, off + h, n - h)


def np_sum_order(x):
    """np.add.reduce over a contiguous float64 array as numpy evaluates it: the
    reduction walks buffers of 8192 elements, r = 0; r += pairwise(buffer)."""
    a = [float(v) for v in np.asarray(x, np.float64).ravel()]
    r = 0.0
    for off in range(0, len(a), 8192):
        r += _np_pairwise(a, off, min(8192, len(a) - off))
    return r


def np_mean_std(x):
    """(np.mean(x), np.std(x)) of a float64 array in numpy's order: mean = sum /
    n; std = sqrt(sum((x - mean) * (x - mean)) / n) (numpy _methods._var)."""
    a = np.asarray(x, np.float64).ravel()
    n = a.size
    mean = np_sum_order(a) / n
    d = a - mean
    return mean, float(np.sqrt(np_sum_order(d * d) / n))


def xcorr_peak(stream, preamble, mode="valid"):
    """Fused form used by the sync stage: correlate + find_correlation_peak.
    Returns (argmax index into the correlation, peak_lag, peak |c|, sum|c|,
    sum|c|^2, confidence) computed in complex128 like the reference."""
    c, lags = cross_correlate_signals(preamble, stream, mode)
    a = np.abs(c)
    i = int(np.argmax(a))
    lag, peak, conf = find_correlation_peak(c, lags)
    return i, int(lag), float(peak), float(a.sum()), float((a * a).sum()), conf


def find_packet_location_in_vector(vector, packet_signal, reference_segment,
                                   search_window=None, correlation_threshold=0.5):
    """utils.py:1372-1434."""
    if search_window is None:
        s0, s1 = 0, len(vector)
    else:
        s0, s1 = search_window
        s0, s1 = max(0, s0), min(len(vector), s1)
    vc, vl = cross_correlate_signals(reference_segment, vector[s0:s1])
    vlag, _, vconf = find_correlation_peak(vc, vl, correlation_threshold)
    pc, pl = cross_correlate_signals(reference_segment, packet_signal)
    plag, _, pconf = find_correlation_peak(pc, pl, correlation_threshold)
    return s0 + vlag - plag, 0, min(vconf, pconf)


def find_packet_start(signal, template=None, threshold_ratio=0.2, window_size=None):
    """utils.py:784-809 (template branch: argmax of |x| (*) |t| 'valid';
    energy branch: boxcar-smoothed |x|^2, median-of-first-10% threshold)."""
    if template is not None:
        c = np.correlate(np.abs(signal), np.abs(template), mode="valid")
        return int(np.argmax(c))
    e = np.abs(signal) ** 2
    if window_size is None:
        window_size = max(1, int(0.02 * len(signal)))
    w = np.ones(max(1, window_size)) / max(1, window_size)
    sm = np.convolve(e, w, mode="same")
    noise = np.median(sm[: len(sm) // 10])
    thr = noise + threshold_ratio * (np.max(sm) - noise)
    idx = np.where(sm >= thr)[0]
    return int(idx[0]) if len(idx) > 0 else 0


def detect_packet_bounds(signal, sample_rate, threshold_ratio=0.2):
    """utils.py:811-825."""
    e = np.abs(signal) ** 2
    w = max(1, int(sample_rate // 1_000_000))
    sm = np.convolve(e, np.ones(w) / w, mode="same")
    noise = np.median(sm[: max(1, len(sm) // 10)])
    thr = noise + threshold_ratio * (sm.max() - noise)
    idx = np.where(sm >= thr)[0]
    if len(idx) == 0:
        return 0, len(signal)
    return idx[0], idx[-1]


# ---------------------------------------------------------------------------
# filter / decimate — reference idioms np.convolve (utils.py:802,816) and
# x[::factor] (utils.py:194).  No reference FIR exists: parity unpinned at the
# reference level, pinned by numpy semantics.
# ---------------------------------------------------------------------------
def fir_filter(x, taps, decim=1):
    """Causal FIR ``np.convolve(x, taps, 'full')[:len(x)]`` then ``[::decim]``."""
    x = np.asarray(x)
    y = np.convolve(x, np.asarray(taps), mode="full")[: len(x)]
    return y[::decim] if decim > 1 else y


def stride_decimate(x, factor):
    """utils.py:192-195 / heavy_packet_optimizer.py:164-168."""
    return np.asarray(x)[::factor]


def pfb_channelize(x, proto, nchan):
    """Critically sampled polyphase filter-bank analysis channelizer
    (BASELINE config 4; no reference counterpart — parity unpinned).
    Nearest reference analogue: the FFT brick-wall channel split
    ``vector_analyzer/split_channels.py:15-44``.

    Windowed pre-sum PFB (C channels, P = len(proto) // C taps per branch):
        z_m[p]  = sum_{q=0}^{P-1} h[q*C + p] * x[m*C + q*C + p]
        y[k, m] = sum_{p=0}^{C-1} z_m[p] * exp(-2j*pi*k*p/C)
    for m = 0 .. (len(x) - P*C) // C.  Output (C, M) complex64, computed here
    in complex128.
    """
    x = np.asarray(x, dtype=np.complex128)
    h = np.asarray(proto, dtype=np.float64)
    C = int(nchan)
    P = len(h) // C
    if P * C != len(h):
        raise ValueError("len(proto) must be a multiple of nchan")
    M = (len(x) - P * C) // C + 1
    if M <= 0:
        return np.zeros((C, 0), np.complex64)
    frames = np.lib.stride_tricks.sliding_window_view(x, P * C)[::C][:M]
    z = (frames * h[None, :]).reshape(M, P, C).sum(axis=1)     # (M, C)
    return np.fft.fft(z, axis=1).T.astype(np.complex64)


# ---------------------------------------------------------------------------
# element-wise steps and formats either side of the chain
# ---------------------------------------------------------------------------
def apply_frequency_shift(signal, freq_shift, sample_rate):
    """utils.py:120-127."""
    if freq_shift == 0:
        return signal
    t = np.arange(len(signal)) / sample_rate
    shift_factor = np.exp(2j * np.pi * freq_shift * t)
    return (signal * shift_factor).astype(np.complex64)


def transplant_packet_in_vector(vector, packet_signal, vector_location, packet_location=0,
                                replace_length=None, normalize_power=True):
    """utils.py:1437-1501 (prints omitted)."""
    new_vector = vector.copy()
    if replace_length is None:
        replace_length = len(packet_signal) - packet_location
    vector_end = min(vector_location + replace_length, len(vector))
    actual_replace_length = vector_end - vector_location
    packet_end = min(packet_location + actual_replace_length, len(packet_signal))
    actual_packet_length = packet_end - packet_location
    if vector_location >= 0 and vector_location < len(vector) and actual_packet_length > 0:
        seg = packet_signal[packet_location:packet_location + actual_packet_length]
        if normalize_power:
            orig = vector[vector_location:vector_location + actual_packet_length]
            op = np.mean(np.abs(orig) ** 2)
            pp = np.mean(np.abs(seg) ** 2)
            if pp > 0 and op > 0:
                seg = seg * np.sqrt(op / pp)
        new_vector[vector_location:vector_location + actual_packet_length] = seg
    return new_vector


def resample_signal(signal, orig_sr, target_sr):
    """utils.py:107-118: scipy.signal.resample(signal, int(len * ratio)) then
    complex64.  Restated from scipy 1.15.3 ``scipy/signal/_signaltools.py``
    resample (domain='time', no window): full FFT (scipy.fft, the input's
    precision), positive bins [0, N//2] and negative bins copied into a
    num-point spectrum, the Nyquist bin split (upsampling) or folded
    (downsampling) for even N = min(num, Nx), inverse FFT, times num / Nx.
    Real input goes through rfft / irfft there; the complex path below gives
    the same values up to rounding, with the imaginary part set to 0."""
    import scipy.fft as sp_fft
    if orig_sr == target_sr:
        return signal
    x = np.asarray(signal)
    num = int(len(x) * (target_sr / orig_sr))
    Nx = x.shape[0]
    real = np.isrealobj(x)
    X = sp_fft.fft(x)
    Y = np.zeros(num, X.dtype)
    N = min(num, Nx)
    nyq = N // 2 + 1
    Y[:nyq] = X[:nyq]
    if N > 2:
        Y[nyq - N:] = X[nyq - N:]
    if N % 2 == 0:
        if num < Nx:
            Y[-N // 2] += X[-N // 2]
        elif Nx < num:
            Y[N // 2] *= 0.5
            Y[num - N // 2] = Y[N // 2]
    y = sp_fft.ifft(Y) * (float(num) / float(Nx))
    if real:
        y = y.real
    return y.astype(np.complex64)


CENTER_FREQ = 5230e6   # vector_analyzer/split_channels.py:7


def filter_channel(data, center_freq, sample_rate, bandwidth):
    """vector_analyzer/split_channels.py:15-44, as written: the frequency axis
    is np.fft.fftfreq(N, 1/sr) * sr + CENTER_FREQ (the extra * sr is the
    reference's own, so the brick-wall mask covers ~|bw / 2| * N / sr**2 bins),
    the masked spectrum's negative half is overwritten by the conjugate mirror
    of its non-negative half (after fftshift; odd N raises numpy's
    broadcasting ValueError), inverse FFT, real part (float64)."""
    n = len(data)
    freqs = np.fft.fftfreq(n, 1 / sample_rate) * sample_rate + CENTER_FREQ
    X = np.fft.fft(data)
    mask = (freqs >= center_freq - bandwidth / 2) & (freqs <= center_freq + bandwidth / 2)
    F = np.zeros_like(X, dtype=complex)
    F[mask] = X[mask]
    neg = np.fft.fftshift(freqs) < CENTER_FREQ
    pos = np.fft.fftshift(freqs) >= CENTER_FREQ
    Fs = np.fft.fftshift(F)
    Fs[neg] = np.conj(np.flip(Fs[pos]))
    return np.real(np.fft.ifft(np.fft.ifftshift(Fs)))


def mat2wv_fields(signal, bNormalize=True):
    """vector_analyzer/mat_to_wv_converter.py:28-50: (interleaved int16 I/Q,
    fRMSdBfs, fPeakPowerdBfs) — the SMU-WV payload and level fields."""
    signal = np.asarray(signal).flatten()
    if bNormalize:
        signal = signal / np.max(np.abs(signal))
        fPeakPowerdBfs = -10 * np.log10(np.max(np.abs(signal) ** 2))
        fRMSdBfs = -10 * np.log10(np.mean(np.abs(signal) ** 2))
    else:
        fPeakPowerdBfs = 0.0
        fRMSdBfs = 0.0
    vicData = signal * 32767
    out = np.empty(2 * signal.size, dtype=np.int16)
    out[0::2] = np.real(vicData).astype(np.int16)
    out[1::2] = np.imag(vicData).astype(np.int16)
    return out, fRMSdBfs, fPeakPowerdBfs


def generate_sample_packet(duration, sr, frequency, amplitude=1.0):
    """utils.py:679-686: a complex128 tone of int(sr * duration) samples."""
    t = np.linspace(0, duration, int(sr * duration), endpoint=False)
    return amplitude * np.exp(2j * np.pi * frequency * t)


def periodic_vector(packet, period_samples, total_samples, start=0):
    """unified_gui.py:1712, 1755-1769: a complex64 vector of total_samples with
    the packet added every period_samples from start, while it fits."""
    vector = np.zeros(total_samples, dtype=np.complex64)
    pos = start
    while pos + len(packet) <= total_samples:
        vector[pos:pos + len(packet)] += packet
        pos += period_samples
    return vector


# ---------------------------------------------------------------------------
# synthetic inputs — SURVEY.md §8(d)
# ---------------------------------------------------------------------------
TONES = ((1.0, 0.05), (0.5, 0.11), (0.25, -0.20))


def synth_iq(n, seed=20250718, chunk=None, offset=0):
    """x[n] = sum_i A_i e^{j 2 pi f_i n} + w[n], w ~ CN(0, 1), complex64."""
    rng = np.random.default_rng(seed if chunk is None else [seed, chunk])
    idx = np.arange(offset, offset + n, dtype=np.float64)
    x = np.zeros(n, np.complex128)
    for a, f in TONES:
        x += a * np.exp(2j * np.pi * f * idx)
    w = (rng.standard_normal(n) + 1j * rng.standard_normal(n)) * np.sqrt(0.5)
    return (x + w).astype(np.complex64)


def qpsk_preamble(L=4096, seed=4096):
    """L QPSK symbols (+-1 +-j)/sqrt(2), complex64."""
    rng = np.random.default_rng(seed)
    b = rng.integers(0, 2, size=(2, L))
    return (((2 * b[0] - 1) + 1j * (2 * b[1] - 1)) / np.sqrt(2)).astype(np.complex64)


def chain_chunk_seconds(args):
    """The bench's CPU baseline for one time chunk (a pool worker: bench.py's
    all-cores cpu_baseline leg maps it over chunks): FIR with
    the chunk's (ntaps-1)-sample left halo, the spectrogram of the filtered
    chunk, the valid correlation over it plus the next chunk's L-1 samples
    (synthesised here: the timing, not the values, is the point) and
    find_correlation_peak.  Returns the seconds the chunk took."""
    import time
    samples, seed, taps, nfft, tmpl, decim = args
    h, L = len(taps) - 1, len(tmpl)
    x = synth_iq(h + samples + (L - 1) * decim, seed=seed)
    t0 = time.perf_counter()
    y = np.convolve(x, taps)[h: h + samples + (L - 1) * decim][::decim]
    spectrum(y[:samples // decim], 1.0, "hann", nfft, 0, nfft)
    c, lags = cross_correlate_signals(tmpl, y, "valid")
    find_correlation_peak(c, lags)
    return time.perf_counter() - t0
