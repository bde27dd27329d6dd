"""The bench's chain (shard.StreamChain with the HIP backend, world 1) at a
test size against the oracle: FIR + decimation, PSD, and the sync peak found
at exactly the planted offset (D = 1 and D = 4, BASELINE configs 2 and 5)."""
import numpy as np
import pytest
import scipy.signal

from oracle import ref

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("decim,L,nfft", [(1, 512, 1024), (4, 512, 1024), (2, 512, 1024),
                                          (1, 4096, 1024), (4, 4096, 1024), (1, 4096, 8192),
                                          (4, 4096, 8192)])
def test_stream_chain_matches_oracle(gpu, decim, L, nfft):
    """L = 4096 runs the bench's correlator (M = 16384, half-frame kernel);
    with nfft = 8192 the PSD runs inside it (vsig_xcorr_exec_psd_dev)."""
    import torch
    from vector_amd.shard import ChainConfig, HipBackend, StreamChain
    n = 1 << 20
    taps = scipy.signal.firwin(255, 0.2).astype(np.float32)
    rng = np.random.default_rng(decim)
    b = rng.integers(0, 2, size=(2, L * decim))
    pre = (((2 * b[0] - 1) + 1j * (2 * b[1] - 1)) / np.sqrt(2)).astype(np.complex64)
    tmpl = np.convolve(pre, taps)[:L * decim][::decim].astype(np.complex64)
    x = ref.synth_iq(n, seed=11)
    k0 = (n // decim // 3) * decim
    x[k0:k0 + L * decim] += 4 * pre
    cfg = ChainConfig(n_local=n, taps=taps, decim=decim, nfft=nfft, template=tmpl)
    ch = StreamChain(cfg, HipBackend(cfg, 0), 0, 1)
    ch.x.copy_(torch.from_numpy(x))
    ch.step()
    torch.cuda.synchronize()
    y = ch.y.cpu().numpy()
    yr = ref.fir_filter(x, taps, decim)
    assert np.abs(y - yr).max() <= 1e-5 * np.abs(yr).max()
    _, _, S = ref.spectrum(yr, 1.0, "hann", nfft, 0, nfft)
    sx = ch.sxx.cpu().numpy().reshape(-1, nfft).T
    den = np.maximum(S.max(axis=0), 1e-30)
    assert (np.abs(sx - S).max(axis=0) / den).max() <= 1e-5
    m, lag, s1, s2, nout = ch.global_peak()
    i, rlag, peak, r1, r2, _ = ref.xcorr_peak(yr, tmpl, "valid")
    assert lag == rlag == k0 // decim
    assert nout == len(yr) - L + 1
    # against the chain's own filtered stream (the oracle's yr differs from it
    # by the FIR's fp32 rounding): the refined max |c| is the exact complex128
    # dot at the lag, the fused sum |c| / sum |c|^2 the fp32 FFT correlation's
    # within north_star's 1e-5 float bar
    _check_peak_on_own_stream(y, tmpl, m, lag, s1, s2)


def _check_peak_on_own_stream(y, tmpl, m, lag, s1, s2):
    L = len(tmpl)
    seg = y[lag: lag + L].astype(np.complex128)
    direct = abs(np.vdot(tmpl.astype(np.complex128), seg))
    assert m == pytest.approx(direct, rel=1e-12)
    # |c| of every output in complex128 (FFT: ~1e-15 of the max, plenty for sums)
    c = np.abs(scipy.signal.correlate(y.astype(np.complex128), tmpl.astype(np.complex128),
                                      "valid", method="fft"))
    assert s1 == pytest.approx(c.sum(), rel=1e-5)
    assert s2 == pytest.approx((c * c).sum(), rel=1e-5)


@pytest.mark.parametrize("decim", [1, 4])
def test_split_first_fir_matches_single_launch(gpu, decim):
    """shard.StreamChain._fir_first (a rank > 0 of a multi-GPU run): the bulk of
    sub-chunk 0 filtered before the left halo lands, the head after it, on the
    HIP backend -- the same filtered stream as one launch over [halo | chunk]."""
    import torch
    from vector_amd.shard import ChainConfig, HipBackend, StreamChain
    n = 1 << 18
    taps = scipy.signal.firwin(255, 0.2).astype(np.float32)
    cfg = ChainConfig(n_local=n, taps=taps, decim=decim, nfft=1024, template=None)
    be = HipBackend(cfg, 0)
    ch = StreamChain(cfg, be, 0, 1)
    h = ch.hist                      # 254 taps' history rounded up to 16: 256
    assert h == 256
    x_ext = torch.from_numpy(ref.synth_iq(n + h, seed=5)).cuda()
    ch.x_ext.copy_(x_ext)
    want = torch.empty(n // decim, dtype=torch.complex64, device="cuda")
    be.fir_into(x_ext[h - 254:], 254, want)          # the minimal history: the same stream
    # the split as _fir_first issues it (exchange skipped: the halo is already in place)
    s = -(-h // decim) * decim
    be.fir_into(ch.x_ext[s: n + h], h, ch.y_ext[s // decim: n // decim])
    be.fir_into(ch.x_ext[: s + h], h, ch.y_ext[: s // decim])
    torch.cuda.synchronize()
    got = ch.y.cpu().numpy()
    w = want.cpu().numpy()
    assert np.abs(got - w).max() <= 1e-5 * np.abs(w).max()


def test_c_example_runs(gpu, tmp_path):
    """examples/chain_c.c: filter -> spectrogram -> sync through the C ABI from
    a C program (child process); exit 0 = the preamble found at its offset."""
    import subprocess
    from test_host_cpu import _build_c_example
    exe = _build_c_example(str(tmp_path / "chain_c"))
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "planted 300001" in r.stdout


def test_stream_chain_long_template(gpu):
    """A 10 000-sample sync template (longer than one correlator chunk): the
    chain's Correlator takes the chunked path; exact lag."""
    import torch
    from vector_amd.shard import ChainConfig, HipBackend, StreamChain
    n, nfft, L = 1 << 20, 1024, 10_000
    taps = scipy.signal.firwin(63, 0.3).astype(np.float32)
    pre = ref.qpsk_preamble(L, seed=31)
    tmpl = np.convolve(pre, taps)[:L].astype(np.complex64)
    x = ref.synth_iq(n, seed=32)
    k0 = 400_003
    x[k0:k0 + L] += pre
    cfg = ChainConfig(n_local=n, taps=taps, decim=1, nfft=nfft, template=tmpl)
    ch = StreamChain(cfg, HipBackend(cfg, 0), 0, 1)
    ch.x.copy_(torch.from_numpy(x))
    ch.step()
    torch.cuda.synchronize()
    yr = ref.fir_filter(x, taps)
    m, lag, s1, s2, nout = ch.global_peak()
    i, rlag, peak, r1, r2, _ = ref.xcorr_peak(yr, tmpl, "valid")
    assert lag == rlag == k0
    _check_peak_on_own_stream(ch.y.cpu().numpy(), tmpl, m, lag, s1, s2)


@pytest.mark.parametrize("decim", [4, 1])
def test_overlapped_refine_back_to_back_steps(gpu, decim):
    """bench.py's default step form (StreamChain overlap_refine): step k's
    refine runs on the context's refine stream beside step k + 1's FIR, which
    writes the other filtered-stream buffer.  Five steps back to back with the
    preamble moved every step, the peak read only after the last one (and,
    joined, after each of the first two): numpy's exact lag every time, the last
    step's filtered stream and peak equal to the plain chain's, and a refine
    fault check (status read) clean.  Then the plain path on the same context
    (the option off again) is exact too."""
    import torch
    from vector_amd.shard import ChainConfig, HipBackend, StreamChain
    n, L = 1 << 20, 4096 // decim
    taps = scipy.signal.firwin(255, 0.2).astype(np.float32)
    pre = ref.qpsk_preamble(L * decim, seed=41)
    tmpl = np.convolve(pre, taps)[: L * decim][::decim].astype(np.complex64)
    base = ref.synth_iq(n, seed=42)
    k0s = [d * decim for d in (1000, 70_001, 123_457, 200_003, 33_333)]
    xs = []
    for k in k0s:
        x = base.copy()
        x[k: k + L * decim] += 3 * pre
        xs.append(torch.from_numpy(x).cuda())
    cfg = ChainConfig(n_local=n, taps=taps, decim=decim, nfft=8192 // decim, template=tmpl)
    be = HipBackend(cfg, 0)
    ch = StreamChain(cfg, be, 0, 1, overlap_refine=True)
    assert ch.overlap and len(ch._y_bufs) == 2
    for s, x in enumerate(xs):
        ch.x.copy_(x)
        ch.step()
        if s < 2:
            assert ch.global_peak()[1] == k0s[s] // decim
    m, lag, s1, s2, nout = ch.global_peak()
    assert lag == k0s[-1] // decim
    be.check_refine()
    y_last = ch.y.cpu().numpy()
    plain = StreamChain(cfg, HipBackend(cfg, 0), 0, 1)
    assert not plain.overlap
    be.set_overlap_refine(False)
    plain.x.copy_(xs[-1])
    plain.step()
    pm = plain.global_peak()
    assert pm[1] == lag and pm[0] == m and pm[2] == s1 and pm[3] == s2
    assert np.array_equal(plain.y.cpu().numpy(), y_last)
