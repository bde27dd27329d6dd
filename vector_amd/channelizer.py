"""Channel splitting: the reference's own channel filter and the config-4
polyphase filter-bank channelizer.

* ``filter_channel`` -- vector_analyzer/split_channels.py:15-44 as written
  (one full-length FFT of any length, brick-wall mask, conjugate mirror,
  inverse FFT, real part), on the any-length transform (bigfft.hip); pinned
  by tests/golden/channel.npz, made from the reference's function.
* ``Channelizer`` / ``pfb_channelize`` -- BASELINE config 4's critically
  sampled windowed-pre-sum PFB (pfb.hip).  It has no reference counterpart;
  its definition is stated in oracle/ref.py (pfb_channelize) and parity is
  against that definition only ("parity unpinned" with respect to the
  reference).
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib
from .dsp import _device_c64, _is_dev, _ptr

__all__ = ["Channelizer", "pfb_channelize", "filter_channel", "CENTER_FREQ"]

CENTER_FREQ = 5230e6   # vector_analyzer/split_channels.py:7


def filter_channel(data, center_freq, sample_rate, bandwidth):
    """split_channels.filter_channel(data, center_freq, sample_rate, bandwidth):
    float64 real signal of len(data).  The mask keeps the bins whose
    ``np.fft.fftfreq(n, 1/sr) * sr + CENTER_FREQ`` (the reference's axis,
    extra ``* sr`` included) lies within center_freq +- bandwidth/2; the
    negative half becomes the conjugate mirror of the masked non-negative
    half.  Odd n > 1 raises ValueError like numpy's shape mismatch does."""
    ctx = _lib.get_context()
    dev = _is_dev(data)
    if dev:
        t = data.to(torch.complex128 if data.dtype in (torch.complex128, torch.float64)
                    else torch.complex64).contiguous()
    else:
        a = np.asarray(data)
        wide = a.dtype in (np.complex128, np.float64) or np.issubdtype(a.dtype, np.integer)
        t = torch.from_numpy(np.ascontiguousarray(a, dtype=np.complex128 if wide else np.complex64)
                             ).to(f"cuda:{ctx.device}")
    n = int(t.numel())
    if n > 1 and n % 2:
        raise ValueError(f"NumPy boolean array indexing assignment cannot assign {(n + 1) // 2} "
                         f"input values to the {(n - 1) // 2} output values where the mask is true")
    y = torch.empty(n, dtype=torch.float64, device=t.device)
    code = "c128" if t.dtype == torch.complex128 else "c64"
    ctx.check(ctx.lib.vsig_filter_channel_dev(ctx.h, _lib.DTYPES[code], _ptr(t), n, float(center_freq),
                                              float(sample_rate), float(bandwidth), _ptr(y)),
              "filter_channel")
    return y if dev else y.cpu().numpy()


class Channelizer:
    """C-channel critically sampled PFB with a fixed real prototype h
    (len(h) = P*C, C in {64, 128, 256}, P in {4, 8, 16}).

    ``ch(x)`` returns Y of shape (C, M), M = (len(x) - P*C)//C + 1, with
    Y[k, m] = sum_p z_m[p] exp(-2j pi k p / C) and
    z_m[p] = sum_q h[q*C + p] x[(m + q)*C + p]  (complex64)."""

    def __init__(self, proto, nchan: int = 64, device: int | None = None):
        h = np.asarray(proto, dtype=np.float32).ravel()
        C = int(nchan)
        if C not in (64, 128, 256):
            raise NotImplementedError("nchan must be 64, 128 or 256")
        if len(h) % C or len(h) // C not in (4, 8, 16):
            raise NotImplementedError("len(proto) must be 4, 8 or 16 times nchan")
        self.ctx = _lib.get_context(device)
        self.nchan, self.ntaps = C, len(h)
        self.h = torch.from_numpy(h).to(f"cuda:{self.ctx.device}")

    def nframes(self, n: int) -> int:
        return max(0, (n - self.ntaps) // self.nchan + 1)

    def __call__(self, x, out: torch.Tensor | None = None):
        ctx = self.ctx
        xd = _device_c64(x, ctx)
        n = int(xd.shape[0])
        M = self.nframes(n)
        if M <= 0:
            e = np.zeros((self.nchan, 0), np.complex64)
            return e if not _is_dev(x) else torch.from_numpy(e).to(xd.device)
        if out is None:
            out = torch.empty((M, self.nchan), dtype=torch.complex64, device=xd.device)
        elif tuple(out.shape) != (M, self.nchan) or out.dtype != torch.complex64 \
                or not out.is_contiguous() or not out.is_cuda:
            raise ValueError(f"out must be a contiguous complex64 CUDA tensor of shape ({M}, "
                             f"{self.nchan}) (frame-major)")
        ctx.bind_stream()
        ctx.check(ctx.lib.vsig_pfb_c64_dev(ctx.h, _ptr(xd), n, _ptr(self.h), self.ntaps,
                                           self.nchan, _ptr(out), M), "pfb")
        if _is_dev(x):
            return out.T
        return out.cpu().numpy().T


def pfb_channelize(x, proto, nchan: int = 64):
    """One-shot form of :class:`Channelizer` (numpy in -> numpy (C, M) out)."""
    return Channelizer(proto, nchan)(x)
