"""Practical HBM ceilings on this box: torch copy, and libvsig's copy probe with
8-B / 16-B lanes and plain / non-temporal stores over 2**28 complex64 (2 GiB
read + 2 GiB written), timed with HIP events; plus a read-only reduction."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import _tune  # noqa: E402,F401  (libvsig_tune.so)
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


res = {}
ms = t(lambda: y.copy_(x))
res["torch_copy"] = (round(ms, 4), round(16 * n / ms / 1e6, 1))
xr = torch.view_as_real(x)
ms = t(lambda: xr.sum())
res["torch_read_sum"] = (round(ms, 4), round(8 * n / ms / 1e6, 1))
import vector_amd as va
from vector_amd import dsp
ctx = va.get_context(0)
ctx.bind_stream()
for v, name in ((0, "probe_8B"), (1, "probe_8B_nt"), (2, "probe_16B"), (3, "probe_16B_nt")):
    for grid in (0, 2048, 16384):
        ms = t(lambda: ctx.check(ctx.lib.vsig_copy_bench(ctx.h, dsp._ptr(x), n, dsp._ptr(y), v, grid), "c"))
        res[f"{name}_g{grid}"] = (round(ms, 4), round(16 * n / ms / 1e6, 1))
for v in range(4, 16):
    U = (2, 4, 8)[(v - 4) // 4]
    name = f"probe_u{U}_16B" + ("_ntl" if v & 2 else "") + ("_nts" if v & 1 else "")
    ms = t(lambda: ctx.check(ctx.lib.vsig_copy_bench(ctx.h, dsp._ptr(x), n, dsp._ptr(y), v, 0), "c"))
    res[name] = (round(ms, 4), round(16 * n / ms / 1e6, 1))
for v in range(16, 28):
    U = (4, 8, 16)[(v - 16) // 4]
    name = f"probe_u{U}_8B" + ("_ntl" if v & 2 else "") + ("_nts" if v & 1 else "")
    ms = t(lambda: ctx.check(ctx.lib.vsig_copy_bench(ctx.h, dsp._ptr(x), n, dsp._ptr(y), v, 0), "c"))
    res[name] = (round(ms, 4), round(16 * n / ms / 1e6, 1))
for v in range(28, 34):
    U = (2, 4, 8)[(v - 28) // 2]
    name = f"read4to1_u{U}" + ("_ntl" if v & 1 else "")
    ms = t(lambda: ctx.check(ctx.lib.vsig_copy_bench(ctx.h, dsp._ptr(x), n, dsp._ptr(y), v, 0), "c"))
    res[name] = (round(ms, 4), round(10 * n / ms / 1e6, 1))   # 8 B read + 2 B written per sample
for v in range(40, 46):       # the same 4:1 pattern with LDS-DMA loads (global_load_lds_dwordx4)
    U = (2, 4, 8)[(v - 40) // 2]
    name = f"read4to1_glds_u{U}" + ("_nt" if v & 1 else "")
    ms = t(lambda: ctx.check(ctx.lib.vsig_copy_bench(ctx.h, dsp._ptr(x), n, dsp._ptr(y), v, 0), "c"))
    res[name] = (round(ms, 4), round(10 * n / ms / 1e6, 1))
for v in range(50, 74):      # 4:1 with the lane width / unroll / both NT policies free
    k = v - 50
    W, U = (8, 4 << ((k % 12) // 4)) if k < 12 else (16, 2 << ((k % 12) // 4))
    name = f"r4w{W}_u{U}" + ("_ntl" if k & 2 else "") + ("_nts" if k & 1 else "")
    ms = t(lambda: ctx.check(ctx.lib.vsig_copy_bench(ctx.h, dsp._ptr(x), n, dsp._ptr(y), v, 0), "c"))
    res[name] = (round(ms, 4), round(10 * n / ms / 1e6, 1))
print(json.dumps(res))
