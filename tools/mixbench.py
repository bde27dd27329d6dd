"""Mixer + FIR: the standalone NCO kernel followed by the FIR, against the
mixer fused into the FIR's loads (2^28 samples, 255 taps, D = 1 and 4)."""
import os
import sys

import numpy as np
import scipy.signal
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import vector_amd as va                      # noqa: E402
from vector_amd import dsp                   # noqa: E402


def timed(fn, it=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it


def main():
    n, fs, sr = 1 << 28, 0.3e9, 2e9
    taps = scipy.signal.firwin(255, 0.2).astype(np.float32)
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.randn(n, dtype=torch.complex64, device="cuda", generator=g)
    for decim in (1, 4):
        f = dsp.FirFilter(taps, decim, 0)
        y = torch.empty(f.out_len(n), dtype=torch.complex64, device="cuda")
        t_mix = timed(lambda: va.apply_frequency_shift(x, fs, sr))
        xm = va.apply_frequency_shift(x, fs, sr)
        t_fir = timed(lambda: f(xm, out=y))
        t_fused = timed(lambda: f(x, out=y, freq_shift=fs, sample_rate=sr))
        t_plain = timed(lambda: f(x, out=y))
        t_fused2 = timed(lambda: f(x, out=y, freq_shift=fs, sample_rate=sr))
        print(f"D={decim}: mixer {t_mix:.3f} ms + FIR {t_fir:.3f} ms = {t_mix + t_fir:.3f} ms; "
              f"fused {t_fused:.3f} / {t_fused2:.3f} ms; FIR alone on the same input {t_plain:.3f} ms",
              flush=True)


if __name__ == "__main__":
    main()
