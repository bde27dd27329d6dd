"""FIR launch time against the relative placement of its input and output
buffers (tuning aid): one 2^28-sample D = 1 (or --decim 4) chain FIR over a
fixed input, the output placed at a sweep of byte offsets inside a larger
buffer; mean ms per launch from the library's HIP-event timer.
  python tools/fir_align.py [decim]"""
import ctypes as C
import os
import sys

import numpy as np
import scipy.signal
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vector_amd import dsp  # noqa: E402

decim = int(sys.argv[1]) if len(sys.argv) > 1 else 1
n = (1 << 28) if decim == 1 else (1 << 31)
taps = scipy.signal.firwin(255, 0.2).astype(np.float32)
fir = dsp.FirFilter(taps, decim, 0)
ctx = fir.ctx
x = torch.randn(n + 254, dtype=torch.complex64, device="cuda")
ny = n // decim
big = torch.empty(ny + (64 << 20) // 8, dtype=torch.complex64, device="cuda")
print("x % 2MB", x.data_ptr() % (2 << 20), "big % 2MB", big.data_ptr() % (2 << 20), flush=True)
for off in [0, 256, 4096, 65536, 1 << 20, 2 << 20, 3 << 20, 4 << 20, 8 << 20, 16 << 20, 32 << 20,
            0, 2 << 20]:
    y = big[off // 8: off // 8 + ny]
    for _ in range(3):
        fir(x, out=y, nhist=254)
    torch.cuda.synchronize()
    ctx.lib.vsig_timing_reset(ctx.h)
    ctx.lib.vsig_timing_enable(ctx.h, 1)
    for _ in range(10):
        fir(x, out=y, nhist=254)
    torch.cuda.synchronize()
    ctx.lib.vsig_timing_enable(ctx.h, 0)
    tot, cnt = C.c_double(), C.c_int64()
    ctx.lib.vsig_timing_read(ctx.h, b"fir", C.byref(tot), C.byref(cnt))
    d = (y.data_ptr() - x.data_ptr()) % (64 << 20)
    print(f"off {off:>9d}  (y - x) mod 64MB {d:>9d}  fir {tot.value / cnt.value:.4f} ms", flush=True)
