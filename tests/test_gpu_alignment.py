"""The 16-byte memory paths and their fallbacks: the FIR's 16-byte segment
loads / stores (pair lane map, load_segment_x4 / fir_store_x4), the PSD's
interleaved 16-byte frame loads and the correlator's launch geometry apply only
when every segment start is 16-byte aligned (a launch-time choice); device
views at odd element offsets, odd tap counts and odd outputs per block take the
8-byte paths.  Both must give the oracle's results."""
import numpy as np
import pytest
import scipy.signal

from oracle import ref

pytestmark = pytest.mark.gpu


def _dev_view(x, off):
    """x as a device tensor view starting `off` complex elements into a buffer
    (off odd: the view is 8- but not 16-byte aligned)."""
    import torch
    buf = torch.zeros(len(x) + off, dtype=torch.complex64, device="cuda")
    v = buf[off:]
    v.copy_(torch.from_numpy(x))
    return v


@pytest.mark.parametrize("decim,ntaps", [(4, 255), (4, 254), (1, 255), (1, 64)])
@pytest.mark.parametrize("off", [0, 1])
def test_fir_aligned_and_misaligned(gpu, decim, ntaps, off):
    import torch
    n = (1 << 17) + 333
    taps = scipy.signal.firwin(ntaps, 0.2).astype(np.float32)
    x = ref.synth_iq(n, seed=ntaps + off)
    xd = _dev_view(x, off)
    y = gpu.filter(xd, taps, decim)
    torch.cuda.synchronize()
    yr = ref.fir_filter(x, taps, decim)
    y = y.cpu().numpy()
    assert y.shape == yr.shape
    assert np.abs(y - yr).max() <= 1e-5 * np.abs(yr).max()


@pytest.mark.parametrize("off", [0, 1])
@pytest.mark.parametrize("hop", [8192, 4097])
def test_psd_8192_aligned_and_misaligned(gpu, off, hop):
    """nfft = nperseg = 8192 with an even hop on an aligned stream runs the
    interleaved 16-byte loads; an odd offset or an odd hop the 8-byte path."""
    import torch
    n = 8192 * 9 + 100
    x = ref.synth_iq(n, seed=7 + off)
    xd = _dev_view(x, off)
    _, _, S = gpu.spectrum(xd, 1.0, "hann", 8192, 8192 - hop, 8192)
    torch.cuda.synchronize()
    _, _, R = ref.spectrum(x, 1.0, "hann", 8192, 8192 - hop, 8192)
    S = S.cpu().numpy() if hasattr(S, "cpu") else S
    assert S.shape == R.shape
    assert (np.abs(S - R).max(axis=0) / R.max(axis=0)).max() <= 1e-5


@pytest.mark.parametrize("off", [0, 1])
@pytest.mark.parametrize("L", [4096, 4095])
def test_correlator_aligned_and_misaligned(gpu, off, L):
    """M = 16384 correlator: even and odd template lengths (hop = M - L + 1
    rounded down to even), aligned and odd-offset streams: exact lag, peak."""
    import torch
    pre = ref.qpsk_preamble(L, seed=L)
    s = ref.synth_iq(70_000, seed=L + off)
    k0 = 33_333
    s[k0:k0 + L] += pre
    sd = _dev_view(s, off)
    lag, val, conf = gpu.correlate_peak(pre, sd, "valid")
    torch.cuda.synchronize()
    want = ref.xcorr_peak(s, pre, "valid")
    assert int(lag) == want[1] == k0
    assert float(val) == pytest.approx(want[2], rel=1e-9)
