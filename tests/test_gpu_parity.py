"""GPU parity: the HIP path (through libvsig.so's C ABI) against the committed
golden fixtures (reference outputs) and the CPU oracle on the same seeded
inputs.

Tolerances (BASELINE.json north_star): index / argmax / lag results bit-exact;
float32 spectra within 1e-5 relative, measured per frame against the frame's
maximum (SURVEY.md §7 hard part (v)); FIR and correlation outputs within 1e-5
of max |reference| (norm-wise: fp32 FFT vs direct-sum numpy / complex128).
"""
import ctypes as C
import glob
import os

import numpy as np
import pytest

from conftest import GOLDEN, golden
from oracle import ref

pytestmark = pytest.mark.gpu

SPEC_TOL = 1e-5
FIR_TOL = 1e-5
XC_TOL = 1e-5


def assert_spectra_close(S, R, tol=SPEC_TOL):
    """per-frame max-normalised error (frames are columns)."""
    S = np.asarray(S, np.float64)
    R = np.asarray(R, np.float64)
    assert S.shape == R.shape
    den = np.maximum(R.max(axis=0), 1e-30)
    err = (np.abs(S - R).max(axis=0) / den).max()
    assert err <= tol, f"spectrum error {err:.3e} > {tol}"


def assert_normwise(y, r, tol):
    y = np.asarray(y)
    r = np.asarray(r)
    assert y.shape == r.shape
    scale = max(np.abs(r).max(), 1e-30)
    err = np.abs(y.astype(np.complex128) - r.astype(np.complex128)).max() / scale
    assert err <= tol, f"error {err:.3e} > {tol}"


# ---------------------------------------------------------------- spectrum
@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "stft_*.npz"))))
def test_spectrum_matches_reference_call(gpu, path):
    g = np.load(path)
    f, t, S = gpu.spectrum(g["x"], 56e6, str(g["window"]), int(g["nperseg"]),
                           int(g["noverlap"]), int(g["nfft"]))
    np.testing.assert_array_equal(f, g["f"])
    np.testing.assert_array_equal(t, g["t"])
    assert S.dtype == np.float32 and S.shape == g["Sxx"].shape
    assert_spectra_close(S, g["Sxx"])


@pytest.mark.parametrize("path", sorted(p for p in glob.glob(os.path.join(GOLDEN, "spec_*.npz"))
                                        if not p.endswith("spec_params.npz")))
def test_create_spectrogram_matches_reference(gpu, path):
    g = np.load(path)
    f, t, S = gpu.create_spectrogram(g["x"], float(g["sr"]))
    assert tuple(S.shape) == tuple(g["shape"])
    np.testing.assert_array_equal(f, g["f"])
    np.testing.assert_array_equal(t, g["t"])
    assert_spectra_close(S[:, g["sel"]], g["Sxx_sel"])
    np.testing.assert_allclose(S.astype(np.float64).sum(axis=0), g["frame_sum"], rtol=1e-5,
                               atol=1e-30)


@pytest.mark.parametrize("nfft", [64, 128, 256, 512, 1024, 2048, 4096, 8192, 16384])
def test_spectrum_all_sizes_vs_oracle(gpu, nfft):
    x = ref.synth_iq(nfft * 9 + 17, seed=nfft)
    nps = nfft - nfft // 8           # zero padding exercised
    f, t, S = gpu.spectrum(x, 2.0, "hann", nps, nps // 3, nfft)
    _, _, R = ref.spectrum(x, 2.0, "hann", nps, nps // 3, nfft)
    assert_spectra_close(S, R)


@pytest.mark.parametrize("nfft,nps,nov", [(100, 100, 0), (1000, 900, 300), (3000, 2500, 1250),
                                          (48, 40, 20), (12_000, 12_000, 6000), (20_001, 9000, 0)])
def test_spectrum_any_nfft_vs_oracle(gpu, nfft, nps, nov):
    """scipy.signal.spectrogram takes any nfft >= nperseg (utils.py:281-291):
    lengths that are not powers of two run as a Bluestein transform per frame
    (in LDS up to 2 nfft - 1 <= 16384, four-step beyond)."""
    x = ref.synth_iq(nfft * 6 + 333, seed=nfft)
    f, t, S = gpu.spectrum(x, 3.0, "hann", nps, nov, nfft)
    fr, tr, R = ref.spectrum(x, 3.0, "hann", nps, nov, nfft)
    np.testing.assert_array_equal(f, fr)
    np.testing.assert_array_equal(t, tr)
    assert_spectra_close(S, R)
    _, _, Ss = gpu.spectrum(x, 3.0, "hann", nps, nov, nfft, fftshift=True)
    assert_spectra_close(Ss, np.fft.fftshift(R, axes=0))


def test_spectrum_window_array_and_shift(gpu):
    x = ref.synth_iq(50_000, seed=9)
    w = np.kaiser(700, 5.0)
    _, _, S = gpu.spectrum(x, 1.0, w, 700, 100, 1024, fftshift=True)
    _, _, R = ref.spectrum(x, 1.0, w, 700, 100, 1024)
    assert_spectra_close(S, np.fft.fftshift(R, axes=0))


def test_spectrum_real_and_double_inputs(gpu):
    rng = np.random.default_rng(4)
    xr = rng.standard_normal(20_000)                         # float64 -> float64 Sxx
    _, _, S = gpu.spectrum(xr, 1.0, "hann", 512, 256, 512)
    _, _, R = ref.spectrum(xr, 1.0, "hann", 512, 256, 512)
    assert S.dtype == R.dtype == np.float64
    assert_spectra_close(S, R)
    x32 = xr.astype(np.float32)
    _, _, S = gpu.spectrum(x32, 1.0, "blackman", 300, 0, 512)
    _, _, R = ref.spectrum(x32, 1.0, "blackman", 300, 0, 512)
    assert S.dtype == R.dtype == np.float32
    assert_spectra_close(S, R)


def test_spectrum_edge_cases(gpu):
    x = ref.synth_iq(1000, seed=1)
    with pytest.warns(UserWarning):                            # nperseg > len -> clipped
        _, _, S = gpu.spectrum(x[:100], 1.0, "hann", 128, 0, 128)
    _, _, R = ref.spectrum(x[:100], 1.0, "hann", 128, 0, 128)
    assert_spectra_close(S, R)
    with pytest.raises(ValueError):
        gpu.spectrum(x, 1.0, "hann", 256, 0, 128)              # nfft < nperseg
    with pytest.raises(ValueError):
        gpu.spectrum(x, 1.0, "hann", 256, 256, 256)            # noverlap >= nperseg
    f, t, S = gpu.spectrum(np.zeros(0, np.complex64), 1.0)
    assert S.size == 0


def test_create_spectrogram_device_tensor_and_stride(gpu):
    import torch
    x = ref.synth_iq(3_000_000, seed=12)                       # > max_samples -> stride 2
    f, t, R = ref.create_spectrogram(x, 56e6)
    fd, td, Sd = gpu.create_spectrogram(torch.from_numpy(x).cuda(), 56e6)
    np.testing.assert_array_equal(fd, f)
    np.testing.assert_array_equal(td, t)
    assert_spectra_close(Sd.cpu().numpy(), R)


def test_reference_spectrogram_tests(gpu):
    """tests/test_utils.py:63-83 of the reference, through vector_amd."""
    sr = 8000
    t = np.linspace(0, 0.1, int(sr * 0.1), endpoint=False)
    sig = np.exp(2j * np.pi * 1000 * t) * np.exp(2j * np.pi * 500 * np.arange(len(t)) / sr)
    f, _, S = gpu.create_spectrogram(sig.astype(np.complex64), sr)
    idx = np.unravel_index(np.argmax(np.abs(S)), S.shape)
    assert abs(f[idx[0]] - 1500) < 2
    f, _, _ = gpu.create_spectrogram(np.zeros(1_500_000, np.float32), 10_000_000)
    assert np.isclose(max(abs(f)), 10_000_000 / 2, rtol=0.01)


# ---------------------------------------------------------------- filter
@pytest.mark.parametrize("nt", [63, 255])
@pytest.mark.parametrize("d", [1, 4])
def test_filter_matches_numpy_golden(gpu, nt, d):
    g = golden("fir.npz")
    y = gpu.filter(g["x"], g[f"taps{nt}"], d)
    assert y.dtype == np.complex64
    assert_normwise(y, g[f"y{nt}_d{d}"], FIR_TOL)


@pytest.mark.parametrize("ntaps", [1, 2, 17, 511, 512, 513, 2048, 4000, 8192])
@pytest.mark.parametrize("decim", [1, 3])
def test_filter_sizes_vs_oracle(gpu, ntaps, decim):
    rng = np.random.default_rng(ntaps)
    x = ref.synth_iq(40_000 + ntaps, seed=ntaps)
    taps = rng.standard_normal(ntaps).astype(np.float32)
    assert_normwise(gpu.filter(x, taps, decim), ref.fir_filter(x, taps, decim), FIR_TOL)


def test_filter_complex_taps_and_short_input(gpu):
    rng = np.random.default_rng(5)
    taps = (rng.standard_normal(40) + 1j * rng.standard_normal(40)).astype(np.complex64)
    for n in (1, 5, 39, 40, 41, 4097):
        x = ref.synth_iq(n, seed=n)
        assert_normwise(gpu.filter(x, taps, 1), ref.fir_filter(x, taps, 1), FIR_TOL)
    with pytest.raises(ValueError):
        gpu.filter(np.zeros(0, np.complex64), taps)


@pytest.mark.parametrize("ntaps,n,decim", [(9000, 30_000, 1), (20_000, 50_000, 4), (16_384, 20_000, 3),
                                           (9000, 100, 1)])
def test_filter_long_taps_vs_oracle(gpu, ntaps, n, decim):
    """np.convolve (utils.py:802, 816) has no length limit: filters over 8192
    taps run as 8192-tap parts summed with their delays."""
    rng = np.random.default_rng(ntaps + n)
    x = ref.synth_iq(n, seed=n)
    taps = (rng.standard_normal(ntaps) / np.sqrt(ntaps)).astype(np.float32)
    assert_normwise(gpu.filter(x, taps, decim), ref.fir_filter(x, taps, decim), FIR_TOL)


@pytest.mark.parametrize("ntaps,nhist,decim", [(9000, 8999, 1), (9000, 3000, 4), (20_000, 19_999, 4),
                                               (20_000, 12_345, 1)])
def test_filter_long_taps_with_history(gpu, ntaps, nhist, decim):
    """The time-chunk form (FirFilter(x, nhist=...), what StreamChain and the
    native chain call per rank) for filters over 8192 taps: the parts' outputs
    are delayed into place past the history.  Against np.convolve over
    [history | chunk] (samples before the history are zeros)."""
    import torch
    rng = np.random.default_rng(ntaps + nhist)
    n = 30_000
    xe = ref.synth_iq(nhist + n, seed=nhist)
    taps = (rng.standard_normal(ntaps) / np.sqrt(ntaps)).astype(np.float32)
    f = gpu.FirFilter(taps, decim)
    y = f(torch.from_numpy(xe).cuda(), nhist=nhist).cpu().numpy()
    want = np.convolve(xe, taps)[nhist: nhist + n][::decim]
    assert_normwise(y, want, FIR_TOL)


def test_filter_real_input_real_output(gpu):
    rng = np.random.default_rng(6)
    x = rng.standard_normal(10_000)
    taps = rng.standard_normal(33)
    y = gpu.filter(x, taps)
    assert y.dtype == np.float64
    assert_normwise(y, np.convolve(x, taps)[: len(x)], FIR_TOL)


# ---------------------------------------------------------------- correlation
def test_cross_correlate_small_golden(gpu):
    g = golden("xcorr_small.npz")
    for mode in ("full", "valid", "same"):
        c, lags = gpu.cross_correlate_signals(g["s1"], g["s2"], mode)
        assert c.dtype == np.complex128
        np.testing.assert_array_equal(lags, g[f"lags_{mode}"])
        assert_normwise(c, g[f"c_{mode}"], XC_TOL)
        if f"peak_{mode}" in g:
            lag, val, conf = gpu.find_correlation_peak(c, lags)
            want = g[f"peak_{mode}"]
            assert lag == want[0]
            assert val == pytest.approx(want[1], rel=1e-5)
            assert conf == pytest.approx(want[2], rel=1e-5, abs=1e-7)
            lag2, val2, conf2 = gpu.correlate_peak(g["s1"], g["s2"], mode)
            assert lag2 == want[0] and val2 == pytest.approx(want[1], rel=1e-5)
            assert conf2 == pytest.approx(want[2], rel=1e-5, abs=1e-7)
        else:
            with pytest.raises(IndexError):
                gpu.find_correlation_peak(c, lags)
            with pytest.raises(IndexError):
                gpu.correlate_peak(g["s1"], g["s2"], mode)


def test_correlate_swapped_lengths_and_small(gpu):
    rng = np.random.default_rng(8)
    for l1, l2 in ((300, 40), (40, 300), (1, 1), (1, 50), (50, 1), (8192, 9000), (9000, 8192)):
        s1 = (rng.standard_normal(l1) + 1j * rng.standard_normal(l1)).astype(np.complex64)
        s2 = (rng.standard_normal(l2) + 1j * rng.standard_normal(l2)).astype(np.complex64)
        for mode in ("full", "valid", "same"):
            c, lags = gpu.cross_correlate_signals(s1, s2, mode)
            r, rl = ref.cross_correlate_signals(s1, s2, mode)
            np.testing.assert_array_equal(lags, rl)
            assert_normwise(c, r, XC_TOL)


def test_correlate_peak_swapped_operands(gpu):
    """signal2 shorter than signal1: np.correlate swaps its operands and
    reverses the output; the fused argmax must index the reversed output
    (ties are broken toward the first reversed index, but the fp32 FFT's
    rounding means flat |c| runs are not exact ties, so none are asserted)."""
    rng = np.random.default_rng(12)
    for l1, l2 in ((300, 40), (5000, 700), (9000, 8192)):
        s1 = (rng.standard_normal(l1) + 1j * rng.standard_normal(l1)).astype(np.complex64)
        s2 = s1[l1 // 3:l1 // 3 + l2].copy()
        lag, val, _ = gpu.correlate_peak(s1, s2, "full")
        r_i, r_lag, r_peak, *_ = ref.xcorr_peak(s2, s1, "full")   # (stream, preamble)
        assert lag == r_lag, (l1, l2, lag, r_lag)
        assert val == pytest.approx(r_peak, rel=1e-5)
        # 'valid' with signal2 shorter: the reference's lag axis is empty
        with pytest.raises(IndexError):
            ref.xcorr_peak(s2, s1, "valid")
        with pytest.raises(IndexError):
            gpu.correlate_peak(s1, s2, "valid")


def test_correlate_peak_4096_preamble(gpu):
    g = golden("xcorr_peak.npz")
    lag, val, conf = gpu.correlate_peak(g["pre"], g["x"], "valid")
    assert lag == int(g["peak_lag"]) == int(g["k0"])
    assert val == pytest.approx(float(g["peak_val"]), rel=1e-5)
    assert conf == pytest.approx(float(g["conf"]), rel=1e-5, abs=1e-7)
    gf = golden("xcorr_peak_full.npz")
    lag, val, conf = gpu.correlate_peak(g["pre"], g["x"], "full")
    assert lag == int(gf["peak_lag"])
    assert val == pytest.approx(float(gf["peak_val"]), rel=1e-5)


def test_find_correlation_peak_exact_argmax(gpu):
    """double-precision reduction: argmax / peak bit-exact vs numpy on complex128."""
    rng = np.random.default_rng(10)
    c = rng.standard_normal(1_000_003) + 1j * rng.standard_normal(1_000_003)
    c[[5, 999_999]] = 50 + 0j                                   # tie: first index wins
    lags = np.arange(len(c)) - 7
    lag, val, conf = gpu.find_correlation_peak(c, lags)
    rl, rv, rc = ref.find_correlation_peak(c, lags)
    assert lag == rl == 5 - 7
    assert val == rv
    assert conf == pytest.approx(rc, abs=1e-9)


def test_find_packet_location(gpu):
    g = golden("packet.npz")
    got = gpu.find_packet_location_in_vector(g["loc_vector"], g["loc_packet"], g["loc_ref"])
    want = g["loc_result"]
    assert got[0] == want[0] and got[1] == want[1]
    assert got[2] == pytest.approx(want[2], rel=1e-5, abs=1e-7)
    got = gpu.find_packet_location_in_vector(g["loc_vector"], g["loc_packet"], g["loc_ref"],
                                             search_window=(10_000, 20_000))
    assert got[0] == g["loc_result_win"][0]


def test_correlator_stream_full_size_property(gpu):
    """C3 shape at 2**26 (reduced from 2**30 to bound test time): the preamble
    planted at k0 must be found exactly; the value must equal the direct dot."""
    import torch
    n, L, k0 = 1 << 26, 4096, 12_345_679
    pre = ref.qpsk_preamble(L)
    g = torch.Generator(device="cuda").manual_seed(5)
    s = torch.randn(n, dtype=torch.complex64, device="cuda", generator=g)
    s[k0:k0 + L] += torch.from_numpy(pre).cuda()
    xc = gpu.Correlator(pre)
    _, pk = xc(s, "valid")
    torch.cuda.synchronize()
    from vector_amd.dsp import _read_peak
    peak, idx, s1, s2 = _read_peak(pk)
    assert idx == k0
    direct = abs(np.vdot(pre.astype(np.complex128), s[k0:k0 + L].cpu().numpy().astype(np.complex128)))
    assert peak == pytest.approx(direct, rel=1e-5)


@pytest.mark.parametrize("ntaps", [255, 300, 1000, 3000])
def test_fir_block_sizes_agree_with_oracle(gpu, ntaps):
    """Every overlap-save FIR block size the library plans (M = 1024 / 4096 /
    8192 / 16384 for these tap counts) against np.convolve, D = 1 and 3."""
    rng = np.random.default_rng(ntaps)
    x = ref.synth_iq(3 * 16384 + 77, seed=ntaps)
    taps = rng.standard_normal(ntaps).astype(np.float32)
    assert_normwise(gpu.filter(x, taps, 1), ref.fir_filter(x, taps, 1), FIR_TOL)
    assert_normwise(gpu.filter(x, taps, 3), ref.fir_filter(x, taps, 3), FIR_TOL)


@pytest.mark.parametrize("L", [1000, 1500, 3000, 4096])
def test_correlator_block_sizes_agree_with_oracle(gpu, L):
    """Correlator block sizes M = 4096 / 8192 / 16384 (L <= 1024 / 2048 /
    8192): general correlation and the streaming Correlator in valid and full
    mode, c stored (out=) and the fused peak record (exact argmax)."""
    import torch
    x = ref.synth_iq(3 * 16384 + 77, seed=L)
    tmpl = ref.qpsk_preamble(L, seed=L)
    c, _ = gpu.cross_correlate_signals(tmpl, x, "valid")
    r, _ = ref.cross_correlate_signals(tmpl, x, "valid")
    assert_normwise(c, r, XC_TOL)
    s = torch.from_numpy(x).cuda()
    xc = gpu.Correlator(tmpl)
    for mode in ("valid", "full"):
        nout = len(x) - L + 1 if mode == "valid" else len(x) + L - 1
        out = torch.empty(nout, dtype=torch.complex64, device="cuda")
        _, pk = xc(s, mode, out=out)
        r, _ = ref.cross_correlate_signals(tmpl, x, mode)
        assert_normwise(out.cpu().numpy(), r, XC_TOL)
        peak, idx, s1, s2 = gpu.dsp._read_peak(pk)
        a = np.abs(r)
        assert idx == int(np.argmax(a))
        assert peak == pytest.approx(a.max(), rel=1e-12)   # refined: fp64 direct sum
        assert s1 == pytest.approx(a.sum(), rel=1e-5)


@pytest.mark.parametrize("decim", [2, 3, 4])
@pytest.mark.parametrize("n", [1, 777, 100_003, 3 * 16384 + 77])
def test_decimating_fir(gpu, decim, n):
    """Decimation folded into the spectrum (M/D-point inverse transforms) for
    D = 2 / 4, the full-rate kernel with the decimating store for D = 3; same
    outputs as np.convolve(x, h)[:n][::D], any length."""
    rng = np.random.default_rng(n + decim)
    x = ref.synth_iq(n, seed=n)
    for taps in (rng.standard_normal(255).astype(np.float32), np.hanning(65)[1:-1].astype(np.float32)):
        assert_normwise(gpu.filter(x, taps, decim), ref.fir_filter(x, taps, decim), FIR_TOL)


@pytest.mark.parametrize("l1,l2", [(20_000, 61_234), (61_234, 20_000), (8193, 30_000),
                                   (16_384, 16_384)])
@pytest.mark.parametrize("mode", ["full", "valid", "same"])
def test_cross_correlate_long_operands(gpu, l1, l2, mode):
    """Both operands longer than 8192 (np.correlate has no limit): the shorter
    one runs as a sum of 8192-sample chunks (one pass each, accumulated in c)."""
    s1 = ref.synth_iq(l1, seed=l1)
    s2 = ref.synth_iq(l2, seed=l2 + 1)
    c, lags = gpu.cross_correlate_signals(s1, s2, mode)
    cr, lr = ref.cross_correlate_signals(s1, s2, mode)
    np.testing.assert_array_equal(lags, lr)
    assert c.dtype == np.complex128 and c.shape == cr.shape
    assert_normwise(c, cr, XC_TOL)


def test_correlate_peak_long_template(gpu):
    """A 20 000-sample QPSK reference planted in a 300 000-sample stream: exact
    lag and peak through the chunked path, fused (no array) and via the array."""
    L, n, k0 = 20_000, 300_000, 123_457
    pre = ref.qpsk_preamble(L, seed=77)
    s = ref.synth_iq(n, seed=78)
    s[k0:k0 + L] += pre
    want = ref.find_correlation_peak(*ref.cross_correlate_signals(pre, s, "valid"))
    got = gpu.correlate_peak(pre, s, "valid")
    assert got[0] == want[0] == k0
    assert got[1] == pytest.approx(want[1], rel=1e-5)
    assert got[2] == pytest.approx(want[2], rel=1e-5, abs=1e-7)
    c, lags = gpu.cross_correlate_signals(pre, s, "valid")
    got2 = gpu.find_correlation_peak(c, lags)
    assert got2[0] == k0
