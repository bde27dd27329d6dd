"""Multi-rank (world_size 2 and 3) CPU test of the time-chunk sharding with the
gloo backend: halos, frame alignment and the global argmax must reproduce the
single-stream result exactly.  Per-rank compute uses the CPU oracle as a
stand-in backend (this test checks the orchestration, not the kernels)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import ref


class OracleBackend:
    """CPU stand-in with HipBackend's interface (test infrastructure)."""

    def __init__(self, cfg):
        self.cfg = cfg

    def empty(self, n, dtype=torch.complex64):
        return torch.zeros(n, dtype=dtype)

    def fir_into(self, x_ext, nhist, y, i0=None):
        x = x_ext.contiguous().numpy()
        if self.cfg.freq_shift:          # apply_frequency_shift at global indices i0 + k
            assert i0 is not None
            t = (i0 + np.arange(len(x))) / self.cfg.sample_rate
            x = (x * np.exp(2j * np.pi * self.cfg.freq_shift * t)).astype(np.complex64)
        full = np.convolve(x, self.cfg.taps)[nhist: len(x)]
        y.copy_(torch.from_numpy(full[:: self.cfg.decim].astype(np.complex64)))

    def psd_into(self, y, sxx):
        _, _, S = ref.spectrum(y.numpy(), 1.0, "hann", self.cfg.nfft, 0, self.cfg.nfft)
        sxx.copy_(torch.from_numpy(np.ascontiguousarray(S.T).ravel()))

    def xcorr_peak(self, s, rec):
        c = np.correlate(s.numpy().astype(np.complex128),
                         self.cfg.template.astype(np.complex128), "valid")
        a = np.abs(c)
        i = int(np.argmax(a))
        rec.copy_(torch.tensor([a[i], 0.0, a.sum(), (a * a).sum()], dtype=torch.float64))
        rec.view(torch.int64)[1] = i


FS, SR = 0.0137, 1.0    # mixer of the freq_shift cases (cycles per sample)


def make_case(world, n_local=4096, decim=2, nfft=256, ntaps=31, L=100, k0=None, freq_shift=0.0):
    rng = np.random.default_rng(world)
    N = world * n_local
    x = ref.synth_iq(N, seed=world)
    taps = rng.standard_normal(ntaps).astype(np.float32)
    pre = ref.qpsk_preamble(L, seed=7)
    if k0 is None:   # straddles the first rank boundary (or a sub-chunk boundary on 1 rank)
        k0 = n_local // decim - L // 2 if world > 1 else n_local // decim // 4 - L // 2
    xm = ref.apply_frequency_shift(x, freq_shift, SR) if freq_shift else x
    y_full = np.convolve(xm, taps)[:N][::decim].astype(np.complex64)
    y_full[k0:k0 + L] += 6 * pre                                   # plant after filtering
    return x, taps, pre, k0, y_full


def _worker(rank, world, port, n_local, decim, nfft, ntaps, L, q, freq_shift=0.0, k0s=None,
            read_every=True):
    """One rank.  k0s: the preamble's global offset at each step (one step per
    entry; default: make_case's single step); read_every: global_peak() after
    every step (else only after the last: the double-buffered all-gather
    records of earlier steps are reused underneath)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from vector_amd.shard import ChainConfig, StreamChain
        x, taps, pre, k0, _ = make_case(world, n_local, decim, nfft, ntaps, L,
                                        freq_shift=freq_shift)
        cfg = ChainConfig(n_local=n_local, taps=taps, decim=decim, nfft=nfft, template=pre,
                          freq_shift=freq_shift, sample_rate=SR)
        plant = [k0]

        class PlantingBackend(OracleBackend):
            """Adds the preamble to the filtered stream at global plant[0] (as the
            single-stream reference does) before the PSD / xcorr stages."""
            def fir_into(self, x_ext, nhist, y, i0=None):
                super().fir_into(x_ext, nhist, y, i0)
                nyk = y.shape[0]
                start = (y.data_ptr() - ch_holder[0].y_ext.data_ptr()) // 8   # offset in the chunk
                lo = rank * (n_local // decim) + start
                hi = lo + nyk
                k = plant[0]
                a, b = max(lo, k), min(hi, k + L)
                if a < b:
                    y[a - lo:b - lo] += torch.from_numpy((6 * pre[a - k:b - k]).astype(np.complex64))

        ch_holder = []
        ch = StreamChain(cfg, PlantingBackend(cfg), rank, world)
        ch_holder.append(ch)
        ch.x.copy_(torch.from_numpy(x[rank * n_local:(rank + 1) * n_local]))
        peaks = []
        steps = k0s if k0s is not None else [k0]
        for j, k in enumerate(steps):
            plant[0] = k
            ch.step()
            if read_every or j == len(steps) - 1:
                peaks.append(ch.global_peak())
        q.put((rank, ch.y.numpy().copy(), ch.sxx.numpy().copy(), peaks))
    finally:
        dist.destroy_process_group()


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(world, n_local, decim, nfft, ntaps, L, freq_shift=0.0, k0s=None, read_every=True):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker,
                         args=(r, world, port, n_local, decim, nfft, ntaps, L, q, freq_shift, k0s,
                               read_every))
             for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, y, sxx, pk = q.get(timeout=120)
        res[r] = (y, sxx, pk)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


@pytest.mark.parametrize("world,decim,L,freq_shift", [
    (2, 2, 100, 0.0), (3, 2, 100, 0.0), (1, 2, 100, 0.0), (2, 1, 100, 0.0), (3, 1, 300, 0.0),
    (2, 1, 450, 0.0), (3, 2, 100, FS), (2, 2, 100, FS),
    (4, 4, 100, 0.0), (8, 4, 100, 0.0), (8, 1, 100, 0.0)])   # the driver's N = 4 / 8 shapes
def test_sharded_chain_matches_single_stream(world, decim, L, freq_shift):
    """decim 1: the left halo's split at ntaps-1 outputs; long templates (L up
    to 450) widen the right halo.  freq_shift: the mixer before the FIR, phase
    from the global sample index on every rank."""
    n_local, nfft, ntaps = 4096, 256, 31
    res = _run(world, n_local, decim, nfft, ntaps, L, freq_shift)
    x, taps, pre, k0, y_full = make_case(world, n_local, decim, nfft, ntaps, L,
                                         freq_shift=freq_shift)
    ny = n_local // decim
    y_cat = np.concatenate([res[r][0] for r in range(world)])
    np.testing.assert_allclose(y_cat, y_full, rtol=0, atol=1e-5 * np.abs(y_full).max())
    _, _, S = ref.spectrum(y_full, 1.0, "hann", nfft, 0, nfft)
    s_cat = np.concatenate([res[r][1] for r in range(world)]).reshape(-1, nfft)
    np.testing.assert_allclose(s_cat, S.T, rtol=1e-5, atol=1e-6 * S.max())
    i, lag, peak, s1, s2, conf = ref.xcorr_peak(y_full, pre, "valid")
    for r in range(world):
        m, gi, a, b, nout = res[r][2][0]
        assert gi == lag == k0                                   # exact, on every rank
        assert nout == world * ny - L + 1
        assert m == pytest.approx(peak, rel=1e-6)
        assert a == pytest.approx(s1, rel=1e-6) and b == pytest.approx(s2, rel=1e-6)


@pytest.mark.parametrize("world,read_every", [(2, True), (3, True), (3, False), (2, False)])
def test_sharded_chain_multi_step_peaks(world, read_every):
    """Five steps with the preamble planted at a different global offset each
    step (on either side of the rank boundaries): the double-buffered,
    asynchronous peak all-gather must give every step's own global peak --
    global_peak() after each step, or only after the last one (the slots of
    earlier steps reused underneath)."""
    n_local, decim, nfft, ntaps, L = 4096, 2, 256, 31, 100
    ny = n_local // decim
    k0s = [ny - L // 2, 300, world * ny - L - 7, ny + 900, 2 * ny // 3]
    res = _run(world, n_local, decim, nfft, ntaps, L, k0s=k0s, read_every=read_every)
    x, taps, pre, _, _ = make_case(world, n_local, decim, nfft, ntaps, L)
    y0 = np.convolve(x, taps)[: world * n_local][::decim].astype(np.complex64)
    want = []
    for k in k0s:
        y = y0.copy()
        y[k:k + L] += 6 * pre
        want.append(ref.xcorr_peak(y, pre, "valid"))
    if not read_every:
        want = want[-1:]
    for r in range(world):
        got = res[r][2]
        assert len(got) == len(want)
        for (m, gi, a, b, nout), w in zip(got, want):
            assert gi == w[1]
            assert m == pytest.approx(w[2], rel=1e-6)
            assert a == pytest.approx(w[3], rel=1e-6)


def test_combine_peaks_tie_lowest_index():
    from vector_amd.shard import combine_peaks
    rows = np.array([(5.0, 900, 1.0, 2.0), (5.0, 100, 1.0, 2.0), (4.0, 3, 1.0, 2.0)], dtype=object)
    m, i, s1, s2 = combine_peaks(rows)
    assert (m, i, s1, s2) == (5.0, 100, 3.0, 6.0)


def test_chain_config_validation():
    from vector_amd.shard import ChainConfig
    with pytest.raises(ValueError):
        ChainConfig(n_local=1000, taps=np.ones(3), decim=3, nfft=64).validate(2)
    with pytest.raises(ValueError):
        ChainConfig(n_local=1024, taps=np.ones(3), decim=1, nfft=1000).validate(2)
    with pytest.raises(ValueError):
        ChainConfig(n_local=128, taps=np.ones(3), nfft=64, template=np.ones(500)).validate(2)


def test_chain_config_fir_halo_boundary():
    """the left halo is ntaps-1 rounded up to 16 (128-byte-aligned
    segment starts), so at world > 1 a chunk must hold that many samples --
    the same bound as chain.hip's vsig_chain_create (ntaps-1 <= n_local < hist
    made the send slice x_ext[n:n+hist] overlap the receive buffer x_ext[:hist])."""
    from vector_amd.shard import ChainConfig, fir_history
    assert fir_history(255) == 256 and fir_history(63) == 64 and fir_history(17) == 16
    assert fir_history(1) == 0 and fir_history(18) == 32
    taps = np.ones(40)                                  # ntaps - 1 = 39 -> hist 48
    ChainConfig(n_local=48, taps=taps, nfft=8).validate(2)
    ChainConfig(n_local=40, taps=taps, nfft=8).validate(1)       # one rank: no halo
    with pytest.raises(ValueError, match="FIR halo"):   # n >= ntaps - 1 but < hist
        ChainConfig(n_local=40, taps=taps, nfft=8).validate(2)


# ---------------------------------------------------------------- sharded PFB (config 4)
class OraclePfbBackend:
    """CPU stand-in for HipPfbBackend (test infrastructure)."""

    def __init__(self, proto, C):
        self.h, self.C = proto, C

    def empty(self, n, dtype=torch.complex64):
        return torch.zeros(n, dtype=dtype)

    def pfb_into(self, x, y):
        Y = ref.pfb_channelize(x.numpy(), self.h, self.C)          # (C, nf)
        y[: Y.size].copy_(torch.from_numpy(np.ascontiguousarray(Y.T).ravel()))


def _pfb_worker(rank, world, port, n_local, C, P, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from vector_amd.shard import PfbChain
        h = np.hanning(P * C).astype(np.float32)
        x = ref.synth_iq(world * n_local, seed=5)
        ch = PfbChain(n_local, h, C, OraclePfbBackend(h, C), rank, world)
        ch.x.copy_(torch.from_numpy(x[rank * n_local:(rank + 1) * n_local]))
        ch.step()
        q.put((rank, ch.frame0, ch.frames().numpy().copy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_pfb_matches_single_stream(world):
    n_local, C, P = 64 * 40, 64, 8
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_pfb_worker, args=(r, world, port, n_local, C, P, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, f0, Y = q.get(timeout=120)
        res[r] = (f0, Y)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    h = np.hanning(P * C).astype(np.float32)
    x = ref.synth_iq(world * n_local, seed=5)
    full = ref.pfb_channelize(x, h, C).T                           # (M, C)
    cat = np.concatenate([res[r][1] for r in range(world)])
    assert cat.shape == full.shape
    np.testing.assert_array_equal(cat, full)
    assert [res[r][0] for r in range(world)] == [r * n_local // C for r in range(world)]
