"""NCO mixer fused into the FIR's loads (vsig_fir_exec_mix_dev, SURVEY.md §8(f)
f2): filter(apply_frequency_shift(x, f, sr)) in one kernel, against the oracle
(utils.py:120-127 restated, then np.convolve + stride) within the FIR
tolerance, on every FIR path (pair kernel D = 1 / 3, frequency-domain
decimation D = 2 / 4), for chunked calls with history and a global phase
origin, and through the chain."""
import numpy as np
import pytest
import scipy.signal

from oracle import ref

pytestmark = pytest.mark.gpu

FIR_TOL = 1e-5
SR, FS = 56e6, 1.5e6


def _close(y, r):
    y = np.asarray(y)
    assert y.shape == r.shape
    err = np.abs(y.astype(np.complex128) - r).max() / np.abs(r).max()
    assert err <= FIR_TOL, f"error {err:.3e}"


@pytest.mark.parametrize("decim", [1, 2, 3, 4])
@pytest.mark.parametrize("ntaps", [63, 255])
def test_filter_with_frequency_shift_vs_oracle(gpu, decim, ntaps):
    n = (1 << 20) + 12_345
    x = ref.synth_iq(n, seed=decim + ntaps)
    taps = scipy.signal.firwin(ntaps, 0.2).astype(np.float32)
    y = gpu.filter(x, taps, decim, freq_shift=FS, sample_rate=SR)
    r = ref.fir_filter(ref.apply_frequency_shift(x, FS, SR), taps, decim)
    _close(y, r)


def test_filter_with_frequency_shift_long_phase(gpu):
    """2^23 samples at sr = 1: |theta| reaches 2^23 * 2 pi * 0.31 (the phase is
    reduced in double before the fp32 rotation)."""
    n = 1 << 23
    x = ref.synth_iq(n, seed=3)
    taps = scipy.signal.firwin(255, 0.3).astype(np.float32)
    y = gpu.filter(x, taps, 1, freq_shift=0.31, sample_rate=1.0)
    r = ref.fir_filter(ref.apply_frequency_shift(x, 0.31, 1.0), taps, 1)
    _close(y, r)


@pytest.mark.parametrize("decim", [1, 4])
def test_chunked_mixed_filter_matches_whole_stream(gpu, decim):
    """Time chunks with their left halo and global phase origin i0 reproduce
    the whole-stream result (the sharded chain's contract)."""
    import torch
    from vector_amd import dsp
    n, nch, ntaps = 1 << 18, 4, 255
    x = ref.synth_iq(n, seed=9)
    taps = scipy.signal.firwin(ntaps, 0.2).astype(np.float32)
    f = dsp.FirFilter(taps, decim, 0)
    xd = torch.from_numpy(x).cuda()
    nk, h = n // nch, ntaps - 1
    parts = []
    for k in range(nch):
        a = k * nk
        lo = max(0, a - h)
        xk = torch.cat([torch.zeros(h - (a - lo), dtype=torch.complex64, device="cuda"),
                        xd[lo: a + nk]])
        parts.append(f(xk, nhist=h, freq_shift=FS, sample_rate=SR, i0=a - h).cpu().numpy())
    r = ref.fir_filter(ref.apply_frequency_shift(x, FS, SR), taps, decim)
    _close(np.concatenate(parts), r)


def test_zero_shift_is_plain_filter(gpu):
    x = ref.synth_iq(50_000, seed=4)
    taps = np.hanning(31).astype(np.float32)
    np.testing.assert_array_equal(gpu.filter(x, taps, 2, freq_shift=0.0, sample_rate=SR),
                                  gpu.filter(x, taps, 2))


@pytest.mark.parametrize("decim", [1, 4])
def test_stream_chain_with_frequency_shift(gpu, decim):
    import torch
    from vector_amd.shard import ChainConfig, HipBackend, StreamChain
    n, nfft, L = 1 << 20, 1024, 512
    taps = scipy.signal.firwin(255, 0.2).astype(np.float32)
    pre = ref.qpsk_preamble(L * decim, seed=5)
    x = ref.synth_iq(n, seed=21)
    k0 = (n // decim // 3) * decim
    x[k0:k0 + L * decim] += 4 * pre
    xm = ref.apply_frequency_shift(x, FS, SR)
    yr = ref.fir_filter(xm, taps, decim)
    tmpl = yr[k0 // decim: k0 // decim + L].copy()
    cfg = ChainConfig(n_local=n, taps=taps, decim=decim, nfft=nfft, template=tmpl,
                      freq_shift=FS, sample_rate=SR)
    ch = StreamChain(cfg, HipBackend(cfg, 0), 0, 1)
    ch.x.copy_(torch.from_numpy(x))
    ch.step()
    torch.cuda.synchronize()
    _close(ch.y.cpu().numpy(), yr)
    m, lag, s1, s2, nout = ch.global_peak()
    assert lag == ref.xcorr_peak(yr, tmpl, "valid")[1] == k0 // decim


def test_long_filter_with_frequency_shift(gpu):
    """ntaps > 256 (4096-point blocks): the standalone mixer runs first, then
    the filter -- the same result contract."""
    n = 300_001
    x = ref.synth_iq(n, seed=8)
    taps = scipy.signal.firwin(400, 0.1).astype(np.float32)
    y = gpu.filter(x, taps, 2, freq_shift=FS, sample_rate=SR)
    r = ref.fir_filter(ref.apply_frequency_shift(x, FS, SR), taps, 2)
    _close(y, r)
