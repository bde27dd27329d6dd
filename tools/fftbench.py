"""FFT engine ceiling: time per point-FFT of each plan without HBM traffic."""
import os, sys, json
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import _tune  # noqa: E402,F401  (libvsig_tune.so)
import vector_amd as va
from vector_amd import dsp
ctx = va.get_context(0)
ctx.bind_stream()
iters = 20
for key in (-1024, 4096, 8192, 16384):
    N = abs(key)
    frames = max(1, (1 << 28) // N // 8)      # 2**25 points per launch
    io = torch.randn(frames * N, dtype=torch.complex64, device="cuda")
    for twl in ((0, 1, 2, 3) if key == 8192 else (0, 1)):
        ctx.check(ctx.lib.vsig_fft_bench(ctx.h, key, dsp._ptr(io), frames, 1, twl), "warm")
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        ctx.check(ctx.lib.vsig_fft_bench(ctx.h, key, dsp._ptr(io), frames, iters, twl), "run")
        e1.record(); torch.cuda.synchronize()
        ms = e0.elapsed_time(e1)
        pts = frames * N * iters
        # equivalent time for 2**28 samples through one FFT of this size
        print(json.dumps(dict(plan=key, twl=twl, ns_per_point=round(ms * 1e6 / pts, 4),
                              ms_per_2p28_fft=round(ms / pts * (1 << 28), 3))), flush=True)
