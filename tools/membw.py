"""Practical HBM ceilings on this box: device copy (read+write) and a read-only
reduction over 2**28 complex64 (2 GiB), timed with HIP events."""
import json
import torch
n = 1 << 28
x = torch.randn(n, dtype=torch.complex64, device="cuda")
y = torch.empty_like(x)
def t(fn, it=20):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it
ms = t(lambda: y.copy_(x))
xr = torch.view_as_real(x)
ms2 = t(lambda: xr.sum())
print(json.dumps({"copy_ms": round(ms, 4), "copy_GBs": round(2 * 8 * n / ms / 1e6, 1),
                  "read_ms": round(ms2, 4), "read_GBs": round(8 * n / ms2 / 1e6, 1)}))
