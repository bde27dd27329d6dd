"""Kernel-variant sweep on one GPU, interleaved rounds in one process
(cdna_hip_programming.md §5.4 rule 24).  Prints ms per launch and GB/s of
algorithmic bytes for each (kernel, variant, block size).

  python tools/tune.py [--samples 2**28] [--rounds 3] [--iters 10]
"""
import argparse
import ctypes as C
import itertools
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import vector_amd as va                      # noqa: E402
from vector_amd import dsp                   # noqa: E402
from vector_amd.windows import get_window   # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--samples", type=int, default=1 << 28)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    n = a.samples
    ctx = va.get_context(0)
    lib, h = ctx.lib, ctx.h
    dev = "cuda:0"
    g = torch.Generator(device=dev).manual_seed(1)
    x = torch.randn(n + 254, dtype=torch.complex64, device=dev, generator=g)
    y = torch.empty(n, dtype=torch.complex64, device=dev)
    sxx = torch.empty(n, dtype=torch.float32, device=dev)
    import scipy.signal
    taps = scipy.signal.firwin(255, 0.2).astype(np.float32)
    tmpl = (np.random.default_rng(0).standard_normal(4096) * (1 + 1j)).astype(np.complex64)
    w = get_window("hann", 8192).astype(np.float32)
    wd = torch.from_numpy(w).to(dev)
    scale = float(1 / w.sum(dtype=np.float64) ** 2)
    pk = torch.zeros(4, dtype=torch.float64, device=dev)

    cases = []
    for v in (16,):
        cases.append(("psd", v, 8192))
    for v, m in itertools.product((8,), (1024,)):
        cases.append(("fir", v, m))
    for v, m in ((10, 16384), (32, 0), (40, 0)):
        cases.append(("xcorr", v, m))
    if a.only:
        cases = [c for c in cases if c[0] in a.only.split(",")]
    objs = {}

    def run(kind, v, m):
        ctx.bind_stream()
        if kind == "psd":
            lib.vsig_set_option(h, b"psd_variant", v)
            rc = lib.vsig_psd_c64_dev(h, dsp._ptr(y), n, 1, dsp._ptr(wd), 8192, 8192, 8192, scale, 0,
                                      dsp._ptr(sxx), n // 8192)
            ctx.check(rc, "psd")
        elif kind == "fir":
            lib.vsig_set_option(h, b"fir_variant", v)
            f = objs[("fir", m)]
            f(x, out=y, nhist=254)
        else:
            lib.vsig_set_option(h, b"xcorr_variant", v)
            xc = objs[("xcorr", m, v & 32)]
            xc(y, "valid", peak=pk)

    for kind, v, m in cases:
        if kind == "fir" and ("fir", m) not in objs:
            lib.vsig_set_option(h, b"fir_m", m)
            objs[("fir", m)] = dsp.FirFilter(taps, 1, 0)
        if kind == "xcorr" and ("xcorr", m, v & 32) not in objs:
            lib.vsig_set_option(h, b"xcorr_m", m)
            lib.vsig_set_option(h, b"xcorr_variant", v)
            objs[("xcorr", m, v & 32)] = dsp.Correlator(tmpl, 0)
    nbytes = {"psd": 12 * n, "fir": 16 * n, "xcorr": 8 * n}
    res = {c: [] for c in cases}
    for r in range(a.rounds):
        for c in cases:
            run(*c)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                run(*c)
            e1.record()
            torch.cuda.synchronize()
            res[c].append(e0.elapsed_time(e1) / a.iters)
    out = []
    for c in cases:
        ms = min(res[c])
        med = sorted(res[c])[len(res[c]) // 2]
        out.append(dict(kernel=c[0], variant=c[1], M=c[2], ms_min=round(ms, 4), ms_med=round(med, 4),
                        GBs=round(nbytes[c[0]] / (ms * 1e-3) / 1e9, 1)))
        print(json.dumps(out[-1]), flush=True)


if __name__ == "__main__":
    main()
