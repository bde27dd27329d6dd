"""The shard classes bench.py runs at --gpus N (vector_amd/shard.py StreamChain
+ HipBackend, PfbChain + HipPfbBackend), on the GPU at world 2 and 3.

Ranks are host threads of one process on cuda:0, one torch stream and one
vsig context each; their exchanges go through NativeTransport over the
library's loopback (the same StreamChain / PfbChain code that bench.py drives
with TorchTransport = torch.distributed over RCCL; only the transport object
differs).  Three steps per rank with the preamble at a different global offset
each step: halo boxes and peak all-gathers are reused across steps.

Against the single-rank chain over the whole capture (SURVEY.md §8(e);
precedent being replaced: heavy_packet_optimizer.py:114-152):
* the global lag is exact on every rank, every step;
* filtered stream and spectra to 1e-5 of their maximum (the overlap-save
  blocks fall differently in a chunk), peak value to 1e-6;
* the PFB's frames equal the single-stream frames (1e-6 of the maximum).
"""
import threading

import numpy as np
import pytest
import scipy.signal
import torch

from oracle import ref

pytestmark = pytest.mark.gpu


def _run_ranks(world, body):
    res, errs = [None] * world, []

    def main(r):
        try:
            st = torch.cuda.Stream()
            with torch.cuda.stream(st):
                res[r] = body(r)
                st.synchronize()
        except Exception as e:      # surfaced below
            import traceback
            errs.append(f"rank {r}: {e!r}\n{traceback.format_exc()}")

    th = [threading.Thread(target=main, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=180)
    assert not any(t.is_alive() for t in th), "a rank thread did not finish"
    assert not errs, errs
    return res


@pytest.mark.parametrize("world,decim,overlap", [(2, 4, False), (3, 4, False), (2, 1, False),
                                                 (4, 4, False), (8, 4, False), (2, 4, True),
                                                 (3, 1, True), (4, 4, True)])
def test_stream_chain_hip_ranks(gpu, world, decim, overlap):
    """overlap: bench.py's default -- each rank's refine on its context's refine
    stream beside its next step's FIR, two filtered-stream buffers, the peak
    all-gather issued behind the refine (StreamChain overlap_refine)."""
    from vector_amd.shard import (ChainConfig, HipBackend, Loopback, NativeTransport,
                                  StreamChain)
    n, L, nfft = 1 << 19, 4096 // decim, 8192 // decim
    N = world * n
    taps = scipy.signal.firwin(255, 0.2).astype(np.float32)
    pre = ref.qpsk_preamble(L * decim, seed=31)
    tmpl = np.convolve(pre, taps)[: L * decim][::decim].astype(np.complex64)
    base = ref.synth_iq(N, seed=32)
    # preamble: straddling the first chunk boundary (its correlation needs the
    # right halo), early in rank 0, late in the last rank
    k0s = [(n // decim - L // 2) * decim, 1000 * decim, (N // decim - L - 50) * decim]
    xs = []
    for k in k0s:
        x = base.copy()
        x[k: k + L * decim] += 3 * pre
        xs.append(torch.from_numpy(x).cuda())

    def cfg(nl):
        return ChainConfig(n_local=nl, taps=taps, decim=decim, nfft=nfft, template=tmpl)

    # the single-rank chain over the whole capture (world 1, no transport)
    whole = StreamChain(cfg(N), HipBackend(cfg(N), 0), 0, 1)
    want = []
    for x in xs:
        whole.x.copy_(x)
        whole.step()
        want.append((whole.y.cpu().numpy(), whole.sxx.cpu().numpy(), whole.global_peak()))
    del whole
    torch.cuda.synchronize()
    lb = Loopback(world)

    def body(r):
        ch = StreamChain(cfg(n), HipBackend(cfg(n), 0), r, world,
                         transport=NativeTransport(lb.transport(r)), overlap_refine=overlap)
        got = []
        for x in xs:
            ch.x.copy_(x[r * n:(r + 1) * n])
            ch.step()
            got.append((ch.y.cpu().numpy(), ch.sxx.cpu().numpy(), ch.global_peak()))
        return got

    res = _run_ranks(world, body)
    for s, (yw, sw, pw) in enumerate(want):
        assert pw[1] == k0s[s] // decim
        y = np.concatenate([res[r][s][0] for r in range(world)])
        sx = np.concatenate([res[r][s][1] for r in range(world)])
        assert np.abs(y - yw).max() <= 1e-5 * np.abs(yw).max()
        assert np.abs(sx - sw).max() <= 1e-5 * sw.max()
        for r in range(world):
            pk = res[r][s][2]
            assert pk[1] == pw[1]                       # exact lag, every rank, every step
            assert pk[0] == pytest.approx(pw[0], rel=1e-6)
            assert pk[4] == pw[4]
            assert pk[2] == pytest.approx(pw[2], rel=1e-5)


@pytest.mark.parametrize("world", [2, 3, 4])
def test_pfb_chain_hip_ranks(gpu, world):
    from vector_amd.shard import HipPfbBackend, Loopback, NativeTransport, PfbChain
    C, P = 64, 16
    n = C * 4096
    N = world * n
    h = np.hanning(P * C).astype(np.float32)
    xs = [torch.from_numpy(ref.synth_iq(N, seed=40 + s)).cuda() for s in range(3)]
    whole = PfbChain(N, h, C, HipPfbBackend(h, C, 0), 0, 1)
    want = []
    for x in xs:
        whole.x.copy_(x)
        whole.step()
        want.append(whole.frames().cpu().numpy())
    del whole
    torch.cuda.synchronize()
    lb = Loopback(world)

    def body(r):
        ch = PfbChain(n, h, C, HipPfbBackend(h, C, 0), r, world,
                      transport=NativeTransport(lb.transport(r)))
        got = []
        for x in xs:
            ch.x.copy_(x[r * n:(r + 1) * n])
            ch.step()
            got.append((ch.frame0, ch.frames().cpu().numpy()))
        return got

    res = _run_ranks(world, body)
    for s, fw in enumerate(want):
        cat = np.concatenate([res[r][s][1] for r in range(world)])
        assert cat.shape == fw.shape
        assert np.abs(cat - fw).max() <= 1e-6 * np.abs(fw).max()
        assert [res[r][s][0] for r in range(world)] == [r * n // C for r in range(world)]
    # and the single-stream frames against the oracle's definition on a slice
    xh = xs[0][: 200 * C + len(h)].cpu().numpy()
    ref_frames = ref.pfb_channelize(xh, h, C).T
    assert np.abs(want[0][: len(ref_frames)] - ref_frames).max() <= 1e-5 * np.abs(ref_frames).max()


def test_rank_diagnostics_world4(gpu):
    """bench.py's per-rank line at world > 1, on the classes it drives: four
    thread ranks (loopback transport) run three timed steps with the stage
    timers (vsig_timing, HIP events per rank context) and the exposed-wait
    events on (StreamChain.enable_wait_timing); bench.rank_row /
    summarize_ranks give every field -- stage min / max over ranks, the
    left- / right-halo and all-gather waits as measured on each rank's stream,
    the rank that set the pace -- and every rank gets the exact lag."""
    import ctypes as C
    import os
    import sys
    import time
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from vector_amd.shard import ChainConfig, HipBackend, Loopback, NativeTransport, StreamChain
    world, decim, n, L = 4, 4, 1 << 19, 1024
    N = world * n
    taps = scipy.signal.firwin(255, 0.2).astype(np.float32)
    pre = ref.qpsk_preamble(L * decim, seed=51)
    tmpl = np.convolve(pre, taps)[: L * decim][::decim].astype(np.complex64)
    x = ref.synth_iq(N, seed=52)
    k0 = (n // decim - L // 2) * decim             # straddles ranks 0 / 1 (right halo)
    x[k0: k0 + L * decim] += 3 * pre
    xt = torch.from_numpy(x).cuda()
    lb = Loopback(world)
    steps = 3

    def body(r):
        cfg = ChainConfig(n_local=n, taps=taps, decim=decim, nfft=2048, template=tmpl)
        be = HipBackend(cfg, 0)
        ch = StreamChain(cfg, be, r, world, transport=NativeTransport(lb.transport(r)))
        ch.x.copy_(xt[r * n:(r + 1) * n])
        ch.step()                                    # warm-up
        torch.cuda.current_stream().synchronize()
        lib, h = be.ctx.lib, be.ctx.h
        lib.vsig_timing_reset(h)
        lib.vsig_timing_enable(h, 1)
        ch.enable_wait_timing(True)
        t0 = time.perf_counter()
        for _ in range(steps):
            ch.step()
        torch.cuda.current_stream().synchronize()
        elapsed = time.perf_counter() - t0
        lib.vsig_timing_enable(h, 0)
        stages = {}
        for k in ("fir", "psd", "xcorr", "refine"):
            tot, cnt = C.c_double(), C.c_int64()
            lib.vsig_timing_read(h, k.encode(), C.byref(tot), C.byref(cnt))
            if cnt.value:
                stages[k] = tot.value / cnt.value
        waits = ch.wait_ms(steps)
        return bench.rank_row(elapsed, steps, stages, waits), ch.global_peak()[1], sorted(waits)

    res = _run_ranks(world, body)
    summ = bench.summarize_ranks([r[0] for r in res])
    print(summ)
    assert all(r[1] == k0 // decim for r in res)
    assert all(r[2] == ["gather", "left_halo", "right_halo"] for r in res)
    assert summ["world"] == world and 0 <= summ["pace_rank"] < world
    for k in bench.RANK_FIELDS:
        assert set(summ[k]) == {"min", "max", "max_rank"}
        assert 0.0 <= summ[k]["min"] <= summ[k]["max"] < 1e4
    for k in ("fir", "psd", "xcorr", "refine"):
        assert summ[k]["min"] > 0.0                  # every rank ran every stage
    assert len(summ["per_rank"]) == world
