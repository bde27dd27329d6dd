"""Parity at BASELINE.json's full sizes and on the branches
the small cases do not reach.

* create_spectrogram's heavy branch (len > 5e6: max_samples <= 1e6,
  time_resolution >= 20 us, hann, nfft <= 1024; utils.py:184-189, 265-276)
  against the oracle on the whole output.
* C2: 2**28 samples through the chain (255-tap FIR, 8192-point PSD, 4096
  template): FIR outputs and PSD frames at sampled positions against the oracle
  run on those slices with their halos, the sync lag exact.
* C3: a 4096-sample preamble over 2**30 samples: exact lag, peak equal to the
  direct double-precision dot product (refined), sums to 1e-5.
* C5 shape (D = 4) at 2**29 samples: decimated FIR / PSD slices and the lag;
  and at the headline's own 2**31 samples per GPU: first / middle / last
  slices (inputs up to index 2**31 - 1) and a preamble planted in the tail.
Inputs are generated on the device (bench.py's generator: tones + CN(0, 1)
noise + the planted preamble); only the checked slices come back to the host.
"""
import os
import sys

import numpy as np
import pytest
import torch

from oracle import ref

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _bench():
    import bench
    return bench


def test_create_spectrogram_heavy_branch(gpu):
    n, sr = 6_000_000, 56e6
    x = ref.synth_iq(n, seed=61)
    p = gpu.spectrogram.spectrogram_params(n, sr)
    assert p["heavy"] and p["window"] == "hann" and p["nfft"] <= 1024 and p["factor"] == 6
    f, t, S = gpu.create_spectrogram(x, sr)
    fr, tr, R = ref.create_spectrogram(x, sr)
    np.testing.assert_array_equal(f, fr)
    np.testing.assert_array_equal(t, tr)
    assert S.shape == R.shape
    err = (np.abs(S.astype(np.float64) - R).max(axis=0) / R.max(axis=0)).max()
    assert err <= 1e-5
    # device input: the stride folded into the kernel's loads
    fd, td, Sd = gpu.create_spectrogram(torch.from_numpy(x).cuda(), sr)
    np.testing.assert_array_equal(Sd.cpu().numpy(), S)


def _chain(gpu, n, decim, seed, k0=None):
    from vector_amd.shard import ChainConfig, HipBackend, StreamChain
    b = _bench()
    taps, pre, tmpl = b.design(255, 4096, decim)
    cfg = ChainConfig(n_local=n, taps=taps, decim=decim, nfft=8192, template=tmpl)
    be = HipBackend(cfg, 0)
    ch = StreamChain(cfg, be, 0, 1)
    if k0 is None:
        k0 = (n // decim // 2 + 12_345) * decim
    b.generate_chunk(ch.x, 0, seed, pre, k0)
    ch.step()
    torch.cuda.synchronize()
    return ch, taps, tmpl, k0


def _check_slices(ch, taps, tmpl, n, decim, starts):
    """FIR outputs [s, s + 8192) (decimated index) and their PSD frame against
    the oracle on x[s*D - 254 .. (s + 8192)*D)."""
    h = len(taps) - 1
    for s in starts:
        lo = s * decim - h
        xs = ch.x[max(lo, 0): (s + 8192) * decim].cpu().numpy()
        if lo < 0:
            xs = np.concatenate([np.zeros(-lo, np.complex64), xs])
        y_ref = np.convolve(xs, taps)[h: h + 8192 * decim][::decim]
        y = ch.y[s: s + 8192].cpu().numpy()
        assert np.abs(y - y_ref).max() <= 1e-5 * np.abs(y_ref).max()
        _, _, R = ref.spectrum(y_ref.astype(np.complex64), 1.0, "hann", 8192, 0, 8192)
        S = ch.sxx[s: s + 8192].cpu().numpy()
        assert np.abs(S - R[:, 0]).max() <= 1e-5 * R.max()


def test_c2_full_size_chain(gpu):
    n = 1 << 28
    ch, taps, tmpl, k0 = _chain(gpu, n, 1, 20250718)
    m, lag, s1, s2, nout = ch.global_peak()
    assert lag == k0
    ny = n
    starts = [0, 8192, ny // 2, ny // 2 + 8192 * 3, ny - 8192 * 7, ny - 8192]
    _check_slices(ch, taps, tmpl, n, 1, starts)
    # the peak against the direct double-precision dot product at the lag
    seg = ch.y[lag: lag + 4096].cpu().numpy().astype(np.complex128)
    direct = abs(np.vdot(tmpl.astype(np.complex128), seg))
    assert m == pytest.approx(direct, rel=1e-12)


def test_c5_shape_decimated_chain(gpu):
    n = 1 << 29
    ch, taps, tmpl, k0 = _chain(gpu, n, 4, 7)
    m, lag, s1, s2, nout = ch.global_peak()
    assert lag == k0 // 4
    ny = n // 4
    _check_slices(ch, taps, tmpl, n, 4, [0, 8192 * 5, ny // 2, ny - 8192])


def test_c5_headline_size_2pow31(gpu):
    """The headline's own per-GPU size (BASELINE configs[4] on one GPU, what
    bench.py times): 2**31 input samples (x_ext = 2**31 + 256 with the FIR
    history, past the 32-bit index range), D = 4.  FIR outputs and PSD frames
    of the first, a middle and the last 8192 decimated outputs against the
    oracle on those input slices with their halos (the last slice reads input
    samples up to 2**31 - 1, x_ext offsets up to 2**31 + 255); a preamble
    planted in the tail of the capture (input sample ~2**31 - 2**18) is found
    at its exact lag, with numpy's |c| (the direct double-precision dot)."""
    n, decim = 1 << 31, 4
    ny = n // decim
    k0 = (ny - 60_001) * decim
    ch, taps, tmpl, k0 = _chain(gpu, n, decim, 2031, k0=k0)
    assert ch.x_ext.numel() > (1 << 31)
    m, lag, s1, s2, nout = ch.global_peak()
    assert lag == k0 // decim
    assert nout == ny - 4096 + 1
    seg = ch.y[lag: lag + 4096].cpu().numpy().astype(np.complex128)
    direct = abs(np.vdot(tmpl.astype(np.complex128), seg))
    assert m == pytest.approx(direct, rel=1e-12)
    _check_slices(ch, taps, tmpl, n, decim, [0, ny // 2 + 8192 * 3, ny - 8192])
    del ch
    torch.cuda.empty_cache()


def test_c3_sync_2pow30(gpu):
    b = _bench()
    n, L, k0 = 1 << 30, 4096, 123_456_789
    _, pre, _ = b.design(255, L)
    x = torch.empty(n, dtype=torch.complex64, device="cuda")
    b.generate_chunk(x, 0, 20250718, pre, k0)
    xc = gpu.Correlator(pre)
    _, pk = xc(x, "valid")
    peak, idx, s1, s2 = gpu.dsp._read_peak(pk)
    assert idx == k0
    seg = x[k0: k0 + L].cpu().numpy().astype(np.complex128)
    direct = abs(np.vdot(pre.astype(np.complex128), seg))
    assert peak == pytest.approx(direct, rel=1e-12)
    # sums over every output against a float64 reduction of a stored |c|
    c = torch.empty(n - L + 1, dtype=torch.complex64, device="cuda")
    xc(x, "valid", out=c)
    a = c.abs().double()
    assert s1 == pytest.approx(float(a.sum()), rel=1e-5)
    assert s2 == pytest.approx(float((a * a).sum()), rel=1e-5)
    del c, a, x
    torch.cuda.empty_cache()


def test_c4_pfb_per_gpu_full_shape(gpu):
    """BASELINE config 4's per-GPU shape: the 64-channel, 16-branch PFB
    (prototype firwin(1024, 1/64), bench.py run_pfb) over 2**29 device-resident
    samples (config 4's 2**31 over 4 GPUs).  Frames at sampled positions (first,
    middle, last, in both walk directions of the kernel's lane groups) against
    the oracle's definition on those input slices, and a tone planted at
    channel 5's centre over the last quarter of the capture lands in channel 5."""
    import scipy.signal
    b = _bench()
    C, P, n = 64, 16, 1 << 29
    proto = scipy.signal.firwin(P * C, 1.0 / C).astype(np.float32)
    x = torch.empty(n, dtype=torch.complex64, device="cuda")
    b.generate_chunk(x, 0, 4242, np.zeros(0, np.complex64), -1)
    q0 = 3 * n // 4
    idx = torch.arange(q0, n, device="cuda", dtype=torch.float64)
    ph = torch.remainder(idx * (5.0 / C), 1.0) * (2 * np.pi)
    x[q0:] += (8.0 * torch.polar(torch.ones_like(ph), ph)).to(torch.complex64)
    del idx, ph
    ch = gpu.Channelizer(proto, C)
    M = ch.nframes(n)
    out = torch.empty((M, C), dtype=torch.complex64, device="cuda")
    ch(x, out=out)
    torch.cuda.synchronize()
    for m0 in (0, 63, 64, 4097, M // 2 - 5, q0 // C + 100, M - 70, M - 8):
        K = 8
        K = min(K, M - m0)
        xs = x[m0 * C: (m0 + K - 1) * C + P * C].cpu().numpy()
        want = ref.pfb_channelize(xs, proto, C).T                 # (K, C)
        got = out[m0: m0 + K].cpu().numpy()
        assert np.abs(got - want).max() <= 1e-5 * np.abs(want).max(), m0
    # the tone: channel 5 holds nearly all the power of the frames inside it
    tail = out[q0 // C + P: q0 // C + P + 4096].abs().pow(2).double().sum(dim=0).cpu().numpy()
    assert int(np.argmax(tail)) == 5
    assert tail[5] > 0.9 * tail.sum()
    del out, x
    torch.cuda.empty_cache()
