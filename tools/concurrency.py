"""Do two HIP streams overlap?  FIR (HBM-bound) on one stream beside the
correlator (VALU-bound) on another, each alone and together (tuning tool)."""
import os
import sys
import time

import numpy as np
import scipy.signal
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vector_amd import dsp, get_context  # noqa: E402


def main():
    n = 1 << 28
    dev = "cuda:0"
    ctx = get_context(0)
    taps = scipy.signal.firwin(255, 0.2).astype(np.float32)
    tmpl = (np.random.default_rng(0).standard_normal(4096) * (1 + 1j)).astype(np.complex64)
    g = torch.Generator(device=dev).manual_seed(1)
    x = torch.randn(n + 254, dtype=torch.complex64, device=dev, generator=g)
    y = torch.empty(n, dtype=torch.complex64, device=dev)
    y2 = torch.randn(n + 4095, dtype=torch.complex64, device=dev, generator=g)
    pk = torch.zeros(4, dtype=torch.float64, device=dev)
    fir = dsp.FirFilter(taps, 1, 0)
    xc = dsp.Correlator(tmpl, 0)
    mode = sys.argv[1] if len(sys.argv) > 1 else "pool"
    if mode == "prio":        # different priority pools
        sa, sb = torch.cuda.Stream(priority=0), torch.cuda.Stream(priority=-1)
    elif mode == "raw":       # fresh HIP streams (own hardware queues while < GPU_MAX_HW_QUEUES)
        import ctypes as C
        hip = C.CDLL("libamdhip64.so")
        hs = []
        for _ in range(2):
            h = C.c_void_p()
            assert hip.hipStreamCreateWithFlags(C.byref(h), 1) == 0
            hs.append(h.value)
        sa, sb = (torch.cuda.ExternalStream(h) for h in hs)
    else:
        sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    print(mode, flush=True)

    def f():
        with torch.cuda.stream(sa):
            fir(x, out=y, nhist=254)

    def c():
        with torch.cuda.stream(sb):
            xc(y2, "valid", peak=pk)

    def timed(fn, it=10):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(it):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / it * 1e3

    for rep in range(2):
        tf = timed(f)
        tc = timed(c)
        tb = timed(lambda: (c(), f()))
        print(f"fir {tf:.3f} ms  xcorr {tc:.3f} ms  sum {tf + tc:.3f}  both {tb:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
