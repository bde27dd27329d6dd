"""Polyphase filter-bank channelizer (BASELINE config 4).

No reference counterpart: the reference splits channels with one full-length
FFT and a brick-wall mask (vector_analyzer/split_channels.py:15-44).  The
build's definition — a critically sampled windowed-pre-sum PFB — is stated in
oracle/ref.py (pfb_channelize) and implemented in pfb.hip; parity is against
that definition only ("parity unpinned" with respect to the reference).
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib
from .dsp import _device_c64, _is_dev, _ptr

__all__ = ["Channelizer", "pfb_channelize"]


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
