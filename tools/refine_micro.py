"""Refine timing micro-benchmark (tuning aid): the fused M = 16384 correlator
(lane keys, as in the chain) over a 2^24-sample stream with a planted 4096-
sample template, repeated; prints the refine status and the mean refine time
from the library's HIP-event timer.  VSIG_LIB selects an A/B build."""
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import vector_amd as va  # noqa: E402

n, L = 1 << 24, 4096
rng = np.random.default_rng(1)
t = ((rng.standard_normal(L) + 1j * rng.standard_normal(L)) / np.sqrt(2)).astype(np.complex64)
x = torch.randn(n, dtype=torch.complex64, device="cuda")
x[n // 3: n // 3 + L] += torch.from_numpy(3 * t).cuda()
xc = va.Correlator(t)
ctx = xc.ctx
for _ in range(5):
    xc(x, "valid")
torch.cuda.synchronize()
ctx.lib.vsig_timing_reset(ctx.h)
ctx.lib.vsig_timing_enable(ctx.h, 1)
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 30):
    _, pk = xc(x, "valid")
torch.cuda.synchronize()
ctx.lib.vsig_timing_enable(ctx.h, 0)
tot, cnt = C.c_double(), C.c_int64()
ctx.lib.vsig_timing_read(ctx.h, b"refine", C.byref(tot), C.byref(cnt))
print(os.environ.get("VSIG_LIB", "base"), "refine", va.dsp.refine_status(ctx),
      f"{tot.value / max(cnt.value, 1) * 1e3:.1f} us", "peak", va.dsp._read_peak(pk)[:2])
