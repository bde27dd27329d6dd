"""Can the HBM-bound D = 4 FIR and the VALU-bound correlator share the GPU?
(tuning build, persistent grids; DESIGN.md §7 'Next').  Config-5 sizes: the
FIR filters 2**31 samples into y1 while the correlator scans an already
filtered y0 (no dependency: the question is only how fast both run at once).
Prints ms for each alone and for both launched together on two streams."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import _tune  # noqa: E402,F401  (libvsig_tune.so)
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from vector_amd import _lib, dsp  # noqa: E402

n = 1 << 31
taps, pre, tmpl = bench.design(255, 4096, 4)
x = torch.empty(n, dtype=torch.complex64, device="cuda")
xr = torch.view_as_real(x)
xr.normal_()
fir = dsp.FirFilter(taps, 4)
xc = dsp.Correlator(tmpl)
y0 = fir(x)
y1 = torch.empty_like(y0)
torch.cuda.synchronize()
ctx = _lib.get_context(0)
sA, sB = torch.cuda.Stream(), torch.cuda.Stream()


def opt(k, v):
    ctx.check(ctx.lib.vsig_set_option(ctx.h, k.encode(), int(v)), k)


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return round(min(ts), 3), round(float(np.median(ts)), 3)


def run_fir():
    fir(x, out=y1)


def run_xc():
    xc(y0)


def both(first):
    cur = torch.cuda.current_stream()
    sA.wait_stream(cur)
    sB.wait_stream(cur)
    order = (("xc", sB, run_xc), ("fir", sA, run_fir))
    if first == "fir":
        order = order[::-1]
    for _, st, fn in order:
        with torch.cuda.stream(st):
            fn()
    cur.wait_stream(sA)
    cur.wait_stream(sB)


res = {}
for fg, xg in ((0, 0), (2048, 256), (1024, 256), (3072, 256), (2048, 512)):
    opt("tune_fir_grid", fg)
    opt("tune_xcorr_grid", xg)
    key = f"fir{fg}_xc{xg}"
    res[key] = {"fir": timed(run_fir), "xcorr": timed(run_xc),
                "both_xc_first": timed(lambda: both("xc")),
                "both_fir_first": timed(lambda: both("fir"))}
    print(key, json.dumps(res[key]), flush=True)
opt("tune_fir_grid", 0)
opt("tune_xcorr_grid", 0)
print(json.dumps(res))
