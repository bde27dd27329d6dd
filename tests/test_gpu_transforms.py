"""Transforms of any length (bigfft.hip: four-step FFT above 16384 points,
Bluestein for every other length) and the reference functions built on them:

* resample_signal (utils.py:107-118, scipy.signal.resample) against
  tests/golden/stream_ops.npz (made by the reference);
* filter_channel (vector_analyzer/split_channels.py:15-44) against
  tests/golden/channel.npz (made by the reference's function, incl. a slice of
  its data/packet_3_bpsk.mat) and its odd-length ValueError;
* the spectrogram with nfft > 16384 (a long window, utils.py:281-291) and
  create_spectrogram parameters that reach it (utils.py:237-268: a large
  time_resolution_us at a high rate).

Tolerance: 1e-5 of max |reference| (complex64 transforms against numpy /
scipy's; the reference's own FFTs are complex64 for complex64 input).
"""
import numpy as np
import pytest
import torch

from conftest import golden
from oracle import ref

pytestmark = pytest.mark.gpu
TOL = 1e-5


def _normwise(y, r):
    y = np.asarray(y).astype(np.complex128)
    r = np.asarray(r).astype(np.complex128)
    assert y.shape == r.shape
    return np.abs(y - r).max() / max(np.abs(r).max(), 1e-300)


def _dft(gpu, x, inverse=False, batch=1):
    ctx = gpu.get_context()
    t = torch.from_numpy(np.ascontiguousarray(x, np.complex64)).cuda()
    y = torch.empty_like(t)
    n = t.numel() // batch
    ctx.check(ctx.lib.vsig_dft_dev(ctx.h, 1, gpu.dsp._ptr(t), n, batch, 1 if inverse else 0, 1,
                                   gpu.dsp._ptr(y)), "dft")
    return y.cpu().numpy()


@pytest.mark.parametrize("n", [1, 2, 3, 7, 100, 1000, 4095, 8192, 12_289, 65_537, 1 << 18,
                               (1 << 20) + 7])
def test_dft_any_length(gpu, n):
    x = ref.synth_iq(n, seed=n)
    assert _normwise(_dft(gpu, x), np.fft.fft(x.astype(np.complex128))) <= TOL
    assert _normwise(_dft(gpu, x, inverse=True), np.fft.ifft(x.astype(np.complex128))) <= TOL


def test_dft_batched(gpu):
    n, b = 3000, 5
    x = ref.synth_iq(n * b, seed=3)
    want = np.fft.fft(x.reshape(b, n).astype(np.complex128), axis=1).ravel()
    assert _normwise(_dft(gpu, x, batch=b), want) <= TOL


@pytest.mark.parametrize("j", range(5))
def test_resample_signal_golden(gpu, j):
    g = golden("stream_ops.npz")
    a, b = g[f"rs{j}_sr"]
    y = gpu.resample_signal(g[f"rs{j}_x"], a, b)
    assert y.dtype == np.complex64 and y.shape == g[f"rs{j}"].shape
    assert _normwise(y, g[f"rs{j}"]) <= TOL


def test_resample_signal_cases(gpu):
    x = ref.synth_iq(5000, seed=8)
    assert gpu.resample_signal(x, 56e6, 56e6) is x                       # utils.py:109-110
    for a, b in ((56e6, 28e6), (20e6, 56e6), (1.0, 3.0), (3.0, 1.0)):   # even / odd N, both ways
        assert _normwise(gpu.resample_signal(x, a, b), ref.resample_signal(x, a, b)) <= TOL
    xr = np.cos(0.01 * np.arange(4096))                                  # real input: rfft path
    y = gpu.resample_signal(xr, 10.0, 25.0)
    r = ref.resample_signal(xr, 10.0, 25.0)
    assert _normwise(y, r) <= TOL and np.all(y.imag == 0)
    yd = gpu.resample_signal(torch.from_numpy(x).cuda(), 56e6, 40e6)     # device in, device out
    assert yd.is_cuda and _normwise(yd.cpu().numpy(), ref.resample_signal(x, 56e6, 40e6)) <= TOL
    with pytest.raises(ValueError):
        gpu.resample_signal(x[:3], 56e6, 10e6)                           # int(3 * 10/56) = 0


@pytest.mark.parametrize("j", range(5))
def test_filter_channel_golden(gpu, j):
    g = golden("channel.npz")
    cf, sr, bw = g[f"args{j}"]
    y = gpu.filter_channel(g[f"x{j}"], cf, sr, bw)
    assert y.dtype == np.float64 and y.shape == g[f"y{j}"].shape
    assert _normwise(y, g[f"y{j}"]) <= TOL


def test_filter_channel_odd_and_device(gpu):
    with pytest.raises(ValueError):
        gpu.filter_channel(ref.synth_iq(1001, seed=45), 5220e6, 56e6, 20e6)
    x = ref.synth_iq(20_000, seed=46)
    yd = gpu.filter_channel(torch.from_numpy(x).cuda(), 5230e6 + 100.0, 800.0, 2e6)
    assert yd.is_cuda
    assert _normwise(yd.cpu().numpy(), ref.filter_channel(x, 5230e6 + 100.0, 800.0, 2e6)) <= TOL


@pytest.mark.parametrize("nfft,nperseg,hop", [(32768, 32768, 32768), (65536, 40_000, 10_000),
                                              (1 << 20, 1 << 20, 1 << 19)])
def test_spectrum_long_frames(gpu, nfft, nperseg, hop):
    x = ref.synth_iq(3 * nfft + 123, seed=nfft)
    _, _, S = gpu.spectrum(x, 1.0, "hann", nperseg, nperseg - hop, nfft)
    _, _, R = ref.spectrum(x, 1.0, "hann", nperseg, nperseg - hop, nfft)
    assert S.shape == R.shape
    err = (np.abs(S.astype(np.float64) - R).max(axis=0) / R.max(axis=0)).max()
    assert err <= TOL


def test_create_spectrogram_long_window(gpu):
    """sr = 300 MHz, time_resolution_us = 20: window 12 000 samples, nfft 32768
    (utils.py:237-268) -- the reference's STFT, not its fallback."""
    x = ref.synth_iq(2_000_000, seed=71)
    p = gpu.spectrogram.spectrogram_params(len(x), 300e6, time_resolution_us=20)
    assert p["nfft"] > 16384
    f, t, S = gpu.create_spectrogram(x, 300e6, time_resolution_us=20)
    fr, tr, R = ref.create_spectrogram(x, 300e6, time_resolution_us=20)
    np.testing.assert_array_equal(f, fr)
    np.testing.assert_array_equal(t, tr)
    err = (np.abs(S.astype(np.float64) - R).max(axis=0) / R.max(axis=0)).max()
    assert err <= TOL
