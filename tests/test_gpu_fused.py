"""Fused filter -> spectrum kernel (firpsd.hip, vsig_fir_psd_exec_dev) against
the oracle: the filtered stream within the FIR tolerance of np.convolve, the
spectrogram of it within the spectrum tolerance of scipy.signal.spectrogram
(nperseg = hop = nfft = 8192, as the chain calls it), for whole, odd and
partial blocks, with and without history, and the frame-aligned split the
sharded chain issues on ranks > 0.  The chain (StreamChain) uses this kernel
with ChainConfig(fuse=True) (bench.py --fuse) for decim 1 / nfft 8192."""
import numpy as np
import pytest
import scipy.signal

from oracle import ref

pytestmark = pytest.mark.gpu

SPEC_TOL = 1e-5
FIR_TOL = 1e-5
NFFT = 8192


def _fused(gpu, x_ext, nhist, taps, shift=0, variant=0):
    import torch
    from vector_amd import dsp, get_context
    from vector_amd.windows import get_window
    ctx = get_context(0)
    ctx.check(ctx.lib.vsig_set_option(ctx.h, b"fir_psd_variant", variant), "set")
    f = dsp.FirFilter(taps, 1, 0)
    assert f.block == 1024
    w = get_window("hann", NFFT).astype(np.float32)
    scale = float(1.0 / float(np.sum(w, dtype=np.float64)) ** 2)
    xd = torch.from_numpy(x_ext).cuda()
    n = len(x_ext) - nhist
    y = torch.full((n,), float("nan"), dtype=torch.complex64, device="cuda")
    sxx = torch.full(((n // NFFT) * NFFT,), float("nan"), dtype=torch.float32, device="cuda")
    f.fir_psd(xd, nhist, y, torch.from_numpy(w).cuda(), NFFT, scale, sxx, shift)
    torch.cuda.synchronize()
    ctx.check(ctx.lib.vsig_set_option(ctx.h, b"fir_psd_variant", 0), "set")
    return y.cpu().numpy(), sxx.cpu().numpy().reshape(-1, NFFT)


def _check(y, sxx, x_ext, nhist, taps, shift=0):
    yr = np.convolve(x_ext, taps)[nhist: len(x_ext)].astype(np.complex64)
    assert np.isfinite(y).all()
    assert np.abs(y - yr).max() <= FIR_TOL * np.abs(yr).max()
    if sxx.shape[0]:
        _, _, S = ref.spectrum(yr, 1.0, "hann", NFFT, 0, NFFT)
        S = S.T
        if shift:
            S = np.fft.fftshift(S, axes=1)
        assert S.shape == sxx.shape
        den = np.maximum(S.max(axis=1), 1e-30)
        err = (np.abs(sxx.astype(np.float64) - S).max(axis=1) / den).max()
        assert err <= SPEC_TOL, f"spectrum error {err:.3e}"


@pytest.mark.parametrize("n,nhist,ntaps", [(3 * 16384, 0, 255), (2 * 16384 + NFFT, 254, 255),
                                           (2 * 16384 + 5000, 0, 63), (100_000, 62, 63),
                                           (5000, 0, 255), (1 << 20, 254, 255)])
def test_fir_psd_fused_vs_oracle(gpu, n, nhist, ntaps):
    taps = scipy.signal.firwin(ntaps, 0.2).astype(np.float32)
    x = ref.synth_iq(n + nhist, seed=n + ntaps)
    y, sxx = _fused(gpu, x, nhist, taps)
    _check(y, sxx, x, nhist, taps)


@pytest.mark.parametrize("variant,shift", [(1, 0), (0, 1)])
def test_fir_psd_fused_nt_stores_and_shift(gpu, variant, shift):
    taps = np.random.default_rng(3).standard_normal(255).astype(np.float32)
    n = 4 * 16384 + 777
    x = ref.synth_iq(n, seed=9)
    y, sxx = _fused(gpu, x, 0, taps, shift=shift, variant=variant)
    _check(y, sxx, x, 0, taps, shift=shift)


def test_fir_psd_fused_unsupported_falls_to_caller(gpu):
    """ntaps > 342 (segments would overlap less than the filter) is refused with
    VSIG_E_UNSUPPORTED: the chain then runs the two stages separately."""
    import torch
    from vector_amd import dsp
    f = dsp.FirFilter(np.ones(400, np.float32), 1, 0)
    x = torch.zeros(NFFT * 2, dtype=torch.complex64, device="cuda")
    y = torch.empty_like(x)
    s = torch.empty(NFFT * 2, dtype=torch.float32, device="cuda")
    w = torch.ones(NFFT, dtype=torch.float32, device="cuda")
    with pytest.raises(Exception):
        f.fir_psd(x, 0, y, w, NFFT, 1.0, s)


def test_fused_frame_split_matches_single_launch(gpu):
    """The split StreamChain._fir_first issues on ranks > 0 when fused: frames
    >= 1 before the left halo lands, frame 0 after it."""
    import torch
    from vector_amd.shard import ChainConfig, HipBackend, StreamChain
    n = 1 << 18
    taps = scipy.signal.firwin(255, 0.2).astype(np.float32)
    cfg = ChainConfig(n_local=n, taps=taps, decim=1, nfft=NFFT, template=None, fuse=True)
    be = HipBackend(cfg, 0)
    ch = StreamChain(cfg, be, 0, 1)
    assert ch.fused
    x_ext = torch.from_numpy(ref.synth_iq(n + 254, seed=5)).cuda()
    ch.x_ext.copy_(x_ext)
    want_y = torch.empty(n, dtype=torch.complex64, device="cuda")
    want_s = torch.empty(n, dtype=torch.float32, device="cuda")
    be.fir_psd_into(x_ext, 254, want_y, want_s)
    s = NFFT
    be.fir_psd_into(ch.x_ext[s: n + 254], 254, ch.y_ext[s: n], ch.sxx[s: n])
    be.fir_psd_into(ch.x_ext[: s + 254], 254, ch.y_ext[: s], ch.sxx[: s])
    torch.cuda.synchronize()
    w = want_y.cpu().numpy()
    assert np.abs(ch.y.cpu().numpy() - w).max() <= 1e-5 * np.abs(w).max()
    ws = want_s.cpu().numpy().reshape(-1, NFFT)
    gs = ch.sxx.cpu().numpy().reshape(-1, NFFT)
    assert (np.abs(gs - ws).max(axis=1) / ws.max(axis=1)).max() <= 1e-5


@pytest.mark.parametrize("fuse", [True, False])
def test_stream_chain_8192_fused_and_unfused(gpu, fuse):
    """The bench's configuration (255 taps, nfft 8192, L 4096) at 2^20 samples."""
    import torch
    from vector_amd.shard import ChainConfig, HipBackend, StreamChain
    n, L = 1 << 20, 4096
    taps = scipy.signal.firwin(255, 0.2).astype(np.float32)
    pre = ref.qpsk_preamble(L, seed=4096)
    tmpl = np.convolve(pre, taps)[:L].astype(np.complex64)
    x = ref.synth_iq(n, seed=12)
    k0 = 300_001
    x[k0:k0 + L] += 4 * pre
    cfg = ChainConfig(n_local=n, taps=taps, decim=1, nfft=NFFT, template=tmpl, fuse=fuse)
    ch = StreamChain(cfg, HipBackend(cfg, 0), 0, 1)
    assert ch.fused == fuse
    ch.x.copy_(torch.from_numpy(x))
    ch.step()
    torch.cuda.synchronize()
    yr = ref.fir_filter(x, taps)
    y = ch.y.cpu().numpy()
    assert np.abs(y - yr).max() <= FIR_TOL * np.abs(yr).max()
    _, _, S = ref.spectrum(yr, 1.0, "hann", NFFT, 0, NFFT)
    sx = ch.sxx.cpu().numpy().reshape(-1, NFFT).T
    assert (np.abs(sx - S).max(axis=0) / np.maximum(S.max(axis=0), 1e-30)).max() <= SPEC_TOL
    m, lag, s1, s2, nout = ch.global_peak()
    i, rlag, peak, r1, r2, _ = ref.xcorr_peak(yr, tmpl, "valid")
    assert lag == rlag == k0
    assert m == pytest.approx(peak, rel=1e-4)
