"""The per-stage clock sinks (vsig_clock_*, include/vsig.h): the effective
shader clock of a kernel family from s_memtime / s_memrealtime stamps of every
64th block, the figure bench.py prints beside each stage's time (stages_ghz).
No reference counterpart (measurement only)."""
import ctypes as C

import numpy as np
import pytest
import scipy.signal
import torch

from oracle import ref

pytestmark = pytest.mark.gpu


def _read(ctx, name):
    ghz, ticks = C.c_double(), C.c_int64()
    ctx.check(ctx.lib.vsig_clock_read(ctx.h, name, C.byref(ghz), C.byref(ticks)), "clock_read")
    return ghz.value, ticks.value


def test_clock_sinks_read_a_plausible_clock_and_leave_results_unchanged(gpu):
    ctx = gpu.get_context()
    taps = scipy.signal.firwin(255, 0.2).astype(np.float32)
    x = torch.from_numpy(ref.synth_iq(1 << 22, seed=3)).cuda()
    fir = gpu.FirFilter(taps, 4)
    want = fir(x).clone()
    ctx.check(ctx.lib.vsig_clock_enable(ctx.h, 1), "clock_enable")
    try:
        for _ in range(3):
            got = fir(x)
        torch.cuda.synchronize()
        ghz, ticks = _read(ctx, b"fir")
    finally:
        ctx.check(ctx.lib.vsig_clock_enable(ctx.h, 0), "clock_disable")
    assert ticks > 0 and 0.3 < ghz < 3.0, (ghz, ticks)
    assert torch.equal(got, want)                  # stamps never touch an output
    # a family that did not run since the enable reads 0
    ctx.check(ctx.lib.vsig_clock_enable(ctx.h, 1), "clock_enable")
    try:
        assert _read(ctx, b"pfb") == (0.0, 0)
    finally:
        ctx.check(ctx.lib.vsig_clock_enable(ctx.h, 0), "clock_disable")
