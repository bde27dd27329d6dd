"""Time-chunk sharding of the streaming chain across GPUs (one process per GPU,
torch.distributed over RCCL/xGMI).

A long capture X of N = world * n samples is split into contiguous chunks;
rank r owns X[r*n, (r+1)*n).  The chain per rank:

  1. left halo   : rank r receives X[r*n - (ntaps-1), r*n) from rank r-1
                   (rank 0 keeps zeros = the causal filter's zero history)
  2. FIR + dec   : y = filter(X)[r*n/D, (r+1)*n/D)          (fir_os kernel)
  3. right halo  : rank r receives y[(r+1)*n/D, + L-1) from rank r+1
  4. PSD         : frames of nfft samples, hop = nfft, never straddling a
                   chunk (n/D is a multiple of nfft)        (psd kernel)
  5. xcorr sync  : valid correlation with the template over [y | halo],
                   fused |c| argmax / sums                   (xcorr_os kernel)
  6. global peak : all_gather of the per-rank (max, index, sums) (32 B/rank)

Outputs are identical to running the chain on the whole stream at once (the
halos carry exactly the samples a chunk boundary needs); only KB-sized halos
and the 32-byte peak records cross xGMI.  Reference precedent: the overlapped
chunking of heavy_packet_optimizer.py:114-152 (whose merge duplicated the
overlap, :195-222 — not reproduced here).

The compute steps go through a backend object so the orchestration can be
unit-tested on CPU with gloo; the product backend is HipBackend (libvsig.so).
"""
from __future__ import annotations

import contextlib
from dataclasses import dataclass

import numpy as np
import torch
import torch.distributed as dist

__all__ = ["ChainConfig", "HipBackend", "StreamChain", "combine_peaks", "HipPfbBackend",
           "PfbChain", "NativeChain", "Loopback"]


@dataclass
class ChainConfig:
    n_local: int                 # input samples per rank
    taps: np.ndarray             # FIR taps (real or complex)
    decim: int = 1
    nfft: int = 8192             # PSD frame = hop (non-overlapping)
    template: np.ndarray | None = None   # sync preamble (None: no xcorr stage)
    window: str = "hann"
    pipeline: int = 1            # sub-chunks per step (FIR / PSD / xcorr overlap on 3 streams)
    serial: bool = False         # sub-chunks in order on one stream: FIR(k+1), PSD(k), xcorr(k)
                                 # (a sub-chunk's filtered samples are re-read while cache-resident)
    freq_shift: float = 0.0      # apply_frequency_shift before the FIR (fused into its loads),
    sample_rate: float = 1.0     # phase from the global sample index (utils.py:120-127)
    one_stream: bool = True      # pipeline == 1: all stages on the caller's stream (the PSD and
                                 # correlator do not overlap anyway; saves the cross-stream waits)

    def validate(self, world: int):
        ny = self.n_local // self.decim
        K = self.pipeline
        if K < 1 or self.n_local % K:
            raise ValueError("n_local must be a multiple of pipeline")
        if self.n_local % (self.decim * K):
            raise ValueError("n_local must be a multiple of decim * pipeline")
        if (ny // K) % self.nfft:
            raise ValueError("n_local/decim/pipeline must be a multiple of nfft (frames never straddle chunks)")
        if self.template is not None and K > 1 and ny // K < len(self.template) - 1:
            raise ValueError("sub-chunk shorter than the template halo")
        if self.template is not None and world > 1 and ny < len(self.template) - 1:
            raise ValueError("chunk shorter than the template halo")
        if world > 1 and self.n_local < len(self.taps) - 1:
            raise ValueError("chunk shorter than the FIR halo")


def combine_peaks(rows: np.ndarray) -> tuple[float, int, float, float]:
    """rows[r] = (max, global index, sum, sum2) -> global record; the largest
    max wins, ties go to the lowest global index (np.argmax's first-max rule)."""
    best = None
    s1 = s2 = 0.0
    for m, i, a, b in rows:
        i = int(i)
        if best is None or m > best[0] or (m == best[0] and i < best[1]):
            best = (float(m), i)
        s1 += float(a)
        s2 += float(b)
    return best[0], best[1], s1, s2


class HipBackend:
    """The product backend: libvsig.so kernels on the rank's GPU."""

    def __init__(self, cfg: ChainConfig, device: int):
        from . import dsp
        from ._lib import get_context
        from .windows import get_window
        self.dsp = dsp
        self.ctx = get_context(device)
        self.dev = torch.device(f"cuda:{device}")
        self.fir = dsp.FirFilter(cfg.taps, cfg.decim, device)
        self.xc = dsp.Correlator(cfg.template, device) if cfg.template is not None else None
        w = get_window(cfg.window, cfg.nfft).astype(np.float32)
        self.win = torch.from_numpy(w).to(self.dev)
        self.scale = float(1.0 / float(np.sum(w, dtype=np.float64)) ** 2)
        self.nfft = cfg.nfft
        self.freq_shift, self.sample_rate = cfg.freq_shift, cfg.sample_rate
        self.lanes = {k: torch.cuda.Stream(device=self.dev) for k in ("fir", "psd", "xcorr")}

    def empty(self, n, dtype=torch.complex64):
        return torch.zeros(n, dtype=dtype, device=self.dev)

    # stream "lanes": the three stages of a pipelined step run on their own
    # HIP streams, ordered by events (FIR(k) -> PSD(k); FIR(k+1) -> xcorr(k)).
    def lane(self, name):
        return torch.cuda.stream(self.lanes[name])

    def record(self):
        ev = torch.cuda.Event()
        ev.record()
        return ev

    def wait(self, ev):
        if ev is not None:
            torch.cuda.current_stream(self.dev).wait_event(ev)

    def join(self):
        cur = torch.cuda.current_stream(self.dev)
        for st in self.lanes.values():
            cur.wait_stream(st)

    def fork(self):
        cur = torch.cuda.current_stream(self.dev)
        for st in self.lanes.values():
            st.wait_stream(cur)

    def fir_into(self, x_ext, nhist, y, i0=0):
        """i0: global sample index of x_ext[0] (the mixer's phase origin)."""
        self.fir(x_ext, out=y, nhist=nhist, freq_shift=self.freq_shift,
                 sample_rate=self.sample_rate, i0=i0)

    def psd_into(self, y, sxx):
        ctx = self.ctx
        ctx.bind_stream()
        n = int(y.shape[0])
        nframes = n // self.nfft
        self.dsp._check_dev(y, n, torch.complex64, "psd input")
        self.dsp._check_dev(sxx, nframes * self.nfft, torch.float32, "psd output")
        ctx.check(ctx.lib.vsig_psd_c64_dev(ctx.h, self.dsp._ptr(y), n, 1, self.dsp._ptr(self.win),
                                           self.nfft, self.nfft, self.nfft, self.scale, 0,
                                           self.dsp._ptr(sxx), nframes), "psd")

    def xcorr_peak(self, s, rec):
        """valid correlation over s into the device float64[4] record rec
        (max |c|, local index (int64 bits), sum |c|, sum |c|^2)."""
        self.xc(s, "valid", peak=rec)


def _lane(be, name):
    return be.lane(name) if hasattr(be, "lane") else contextlib.nullcontext()


def _record(be):
    return be.record() if hasattr(be, "record") else None


def _wait(be, ev):
    if hasattr(be, "wait"):
        be.wait(ev)


class StreamChain:
    """One rank's part of the sharded chain (world = 1: the plain chain)."""

    def __init__(self, cfg: ChainConfig, backend, rank: int = 0, world: int = 1, group=None):
        cfg.validate(world)
        self.cfg, self.be, self.rank, self.world, self.group = cfg, backend, rank, world, group
        self.hist = len(cfg.taps) - 1
        self.ny = cfg.n_local // cfg.decim
        self.L = len(cfg.template) if cfg.template is not None else 0
        self.yhalo = (self.L - 1) if (self.L and rank < world - 1) else 0
        self.x_ext = backend.empty(self.hist + cfg.n_local)          # [left halo | chunk]
        self.y_ext = backend.empty(self.ny + max(self.L - 1, 0))     # [chunk out | right halo]
        self.sxx = backend.empty((self.ny // cfg.nfft) * cfg.nfft, torch.float32)
        # peak records, double-buffered: the all-gather of step k runs behind
        # step k + 1 (it is waited for only before step k + 2 reuses its slot,
        # or by global_peak); every rank's records land in place (no copies)
        K = cfg.pipeline
        self._recs = backend.empty(2 * 4 * K, torch.float64).view(2, K, 4)
        self._rows = backend.empty(2 * 4 * K * world, torch.float64).view(2, world * K, 4)
        self._gather = [None, None]
        self._slot = 1
        self.peak_rows = None

    @property
    def x(self):
        """The rank's own input chunk (fill it before step())."""
        return self.x_ext[self.hist:]

    @property
    def y(self):
        return self.y_ext[: self.ny]

    @property
    def recs(self):
        """This step's peak records (one per sub-chunk)."""
        return self._recs[self._slot]

    def _begin_step(self):
        self._slot ^= 1
        work, self._gather[self._slot] = self._gather[self._slot], None
        if work is not None:              # the all-gather two steps back (long done)
            work.wait()

    def _gather_peaks(self):
        rows = self._rows[self._slot]
        self._gather[self._slot] = dist.all_gather_into_tensor(rows, self.recs, group=self.group,
                                                               async_op=True)
        return list(rows.view(self.world, self.cfg.pipeline, 4).unbind(0))

    def _exchange_start(self, send, dst, recv, src):
        ops = []
        if send is not None and dst is not None:
            ops.append(dist.P2POp(dist.isend, send, dst, group=self.group))
        if recv is not None and src is not None:
            ops.append(dist.P2POp(dist.irecv, recv, src, group=self.group))
        return dist.batch_isend_irecv(ops) if ops else []

    @staticmethod
    def _exchange_wait(reqs):
        for req in reqs:
            req.wait()

    def _exchange(self, send, dst, recv, src):
        self._exchange_wait(self._exchange_start(send, dst, recv, src))

    def _fir(self, be, a, b, y):
        """FIR of the rank's input samples [a, b) (plus their history) into y."""
        x = self.x_ext[a: b + self.hist]
        if self.cfg.freq_shift:
            be.fir_into(x, self.hist, y, self.rank * self.cfg.n_local - self.hist + a)
        else:
            be.fir_into(x, self.hist, y)

    def _fir_first(self, be, nk, nyk):
        """FIR of sub-chunk 0 with the left-halo exchange hidden behind it:
        outputs from a decimation-aligned s >= ntaps-1 on need only the rank's
        own samples and are filtered while the halo is in flight; the first
        s outputs follow once it has landed."""
        r, w, hist, n = self.rank, self.world, self.hist, self.cfg.n_local
        D = self.cfg.decim

        def run(a, b):
            self._fir(be, a, b, self.y_ext[a // D: b // D])
        if not (w > 1 and hist > 0):
            run(0, nk)
            return
        reqs = self._exchange_start(self.x_ext[n: n + hist] if r < w - 1 else None,
                                    r + 1 if r < w - 1 else None,
                                    self.x_ext[: hist] if r > 0 else None,
                                    r - 1 if r > 0 else None)
        s = -(-hist // D) * D
        if s < nk:
            run(s, nk)
        self._exchange_wait(reqs)
        run(0, min(s, nk))

    def step(self):
        self._begin_step()
        if self.cfg.serial:
            return self._step_serial()
        if self.cfg.pipeline == 1 and self.cfg.one_stream:
            return self._step_single()
        r, w, K = self.rank, self.world, self.cfg.pipeline
        be = self.be
        n, hist, ny, L = self.cfg.n_local, self.hist, self.ny, self.L
        nk, nyk = n // K, ny // K
        if hasattr(be, "fork"):
            be.fork()
        ev_fir, ev_halo = [], None
        with _lane(be, "fir"):
            for k in range(K):                  # 1-2. left halo + FIR (+ decimation), sub-chunk k
                if k == 0:
                    self._fir_first(be, nk, nyk)
                else:
                    self._fir(be, k * nk, (k + 1) * nk, self.y_ext[k * nyk: (k + 1) * nyk])
                ev_fir.append(_record(be))
                if k == 0 and w > 1 and L > 1:  # 3. right halo of the filtered stream
                    self._exchange(self.y_ext[: L - 1] if r > 0 else None,
                                   r - 1 if r > 0 else None,
                                   self.y_ext[ny: ny + L - 1] if r < w - 1 else None,
                                   r + 1 if r < w - 1 else None)
                    ev_halo = _record(be)
        for k in range(K):
            with _lane(be, "psd"):              # 4. PSD of sub-chunk k
                _wait(be, ev_fir[k])
                be.psd_into(self.y_ext[k * nyk: (k + 1) * nyk], self.sxx[k * nyk: (k + 1) * nyk])
            if L:                               # 5. sync correlation of sub-chunk k
                with _lane(be, "xcorr"):
                    last = k == K - 1
                    _wait(be, ev_fir[k + 1] if not last else ev_fir[k])
                    if last and ev_halo is not None:
                        _wait(be, ev_halo)
                    halo = (L - 1) if (not last or r < w - 1) else 0
                    be.xcorr_peak(self.y_ext[k * nyk: (k + 1) * nyk + halo], self.recs[k])
        if hasattr(be, "join"):
            be.join()
        if L:
            if w > 1:                           # 6. global peak records
                self.peak_rows = self._gather_peaks()
            else:
                self.peak_rows = [self.recs]

    def _step_single(self):
        """One sub-chunk, every stage on the current stream: FIR (left halo
        hidden behind its bulk), the right-halo exchange started behind it,
        the PSD while the halo is in flight, then the correlator once it has
        landed, then the peak records."""
        r, w, n, ny, L = self.rank, self.world, self.cfg.n_local, self.ny, self.L
        be = self.be
        self._fir_first(be, n, ny)
        reqs = []
        if w > 1 and L > 1:
            reqs = self._exchange_start(self.y_ext[: L - 1] if r > 0 else None,
                                        r - 1 if r > 0 else None,
                                        self.y_ext[ny: ny + L - 1] if r < w - 1 else None,
                                        r + 1 if r < w - 1 else None)
        be.psd_into(self.y_ext[: ny], self.sxx)
        if L:
            self._exchange_wait(reqs)
            halo = (L - 1) if r < w - 1 else 0
            be.xcorr_peak(self.y_ext[: ny + halo], self.recs[0])
            if w > 1:
                self.peak_rows = self._gather_peaks()
            else:
                self.peak_rows = [self.recs]
        else:
            self._exchange_wait(reqs)

    def _step_serial(self):
        """The same step with the sub-chunks run in order on the current stream,
        PSD(k) and xcorr(k) right after FIR(k+1) (xcorr(k) needs the first L-1
        filtered samples of sub-chunk k+1): each sub-chunk's filtered stream is
        re-read soon after it is written instead of a whole chunk later."""
        r, w, K = self.rank, self.world, self.cfg.pipeline
        be = self.be
        n, hist, ny, L = self.cfg.n_local, self.hist, self.ny, self.L
        nk, nyk = n // K, ny // K

        def fir(k):
            if k == 0:                          # with the left-halo exchange
                self._fir_first(be, nk, nyk)
                return
            self._fir(be, k * nk, (k + 1) * nk, self.y_ext[k * nyk: (k + 1) * nyk])

        def consume(k):
            be.psd_into(self.y_ext[k * nyk: (k + 1) * nyk], self.sxx[k * nyk: (k + 1) * nyk])
            if L:
                last = k == K - 1
                halo = (L - 1) if (not last or r < w - 1) else 0
                be.xcorr_peak(self.y_ext[k * nyk: (k + 1) * nyk + halo], self.recs[k])

        fir(0)
        if w > 1 and L > 1:                     # right halo of the filtered stream
            self._exchange(self.y_ext[: L - 1] if r > 0 else None,
                           r - 1 if r > 0 else None,
                           self.y_ext[ny: ny + L - 1] if r < w - 1 else None,
                           r + 1 if r < w - 1 else None)
        for k in range(1, K):
            fir(k)
            consume(k - 1)
        consume(K - 1)
        if L:
            if w > 1:
                self.peak_rows = self._gather_peaks()
            else:
                self.peak_rows = [self.recs]

    def global_peak(self):
        """(max |c|, global lag, sum |c|, sum |c|^2, n_outputs) of the last step."""
        work = self._gather[self._slot]
        if work is not None:
            work.wait()
        rows = []
        nyk = self.ny // self.cfg.pipeline
        for r, t in enumerate(self.peak_rows):
            h = t.detach().cpu().reshape(-1, 4)
            hi = h.view(torch.int64)
            for k in range(h.shape[0]):
                idx = int(hi[k, 1].item())
                rows.append((float(h[k, 0]), r * self.ny + k * nyk + idx, float(h[k, 2]),
                             float(h[k, 3])))
        m, i, s1, s2 = combine_peaks(np.array(rows, dtype=object))
        nout = self.world * self.ny - self.L + 1
        return m, i, s1, s2, nout


# ---------------------------------------------------------------------------
# The same shard as one native object (C ABI vsig_chain_*, chain.hip)
# ---------------------------------------------------------------------------
class Loopback:
    """In-process loopback transport (vsig_loopback_*): ranks as threads of one
    process, halos copied device to device (tests run several ranks on one GPU)."""

    def __init__(self, world: int):
        import ctypes as C
        from ._lib import load_library
        self.lib = load_library()
        h = C.c_void_p()
        rc = self.lib.vsig_loopback_create(int(world), C.byref(h))
        if rc:
            raise ValueError(f"vsig_loopback_create: {rc}")
        self.h, self.world = h, world

    def transport(self, rank: int):
        import ctypes as C
        from ._lib import Transport
        t = Transport()
        rc = self.lib.vsig_loopback_transport(self.h, int(rank), C.byref(t))
        if rc:
            raise ValueError(f"vsig_loopback_transport: {rc}")
        return t

    def __del__(self):
        try:
            if self.h:
                self.lib.vsig_loopback_free(self.h)
                self.h = None
        except Exception:
            pass


class NativeChain:
    """One rank of the time-chunk shard as a native vsig_chain: the same
    stages, halos and global peak as StreamChain, driven by C++ (chain.hip)
    through a vsig_transport (RCCL communicator, or Loopback for ranks in one
    process).  Enqueues on the calling thread's context stream."""

    def __init__(self, cfg: ChainConfig, device: int, rank: int = 0, world: int = 1, transport=None):
        import ctypes as C
        from ._lib import ChainConfig as CCfg, get_context
        from .windows import get_window
        cfg.validate(world)
        self.ctx = get_context(device)
        self.cfg, self.rank, self.world = cfg, rank, world
        taps = np.ascontiguousarray(np.asarray(cfg.taps).ravel(), dtype=np.complex64)
        w = get_window(cfg.window, cfg.nfft).astype(np.float32)
        tm = (np.ascontiguousarray(np.asarray(cfg.template).ravel(), dtype=np.complex64)
              if cfg.template is not None else None)
        self._keep = (taps, w, tm, transport)
        cc = CCfg(n_local=cfg.n_local, taps=taps.ctypes.data, ntaps=len(taps), decim=cfg.decim,
                  nfft=cfg.nfft, window=w.ctypes.data,
                  psd_scale=float(1.0 / float(np.sum(w, dtype=np.float64)) ** 2),
                  tmpl=tm.ctypes.data if tm is not None else None,
                  L=len(tm) if tm is not None else 0)
        h = C.c_void_p()
        self.ctx.check(self.ctx.lib.vsig_chain_create(self.ctx.h, C.byref(cc), rank, world,
                                                      C.byref(transport) if transport is not None
                                                      else None, C.byref(h)), "vsig_chain_create")
        self.h = h
        self.ny = cfg.n_local // cfg.decim
        self.L = len(tm) if tm is not None else 0

    def load(self, x: torch.Tensor):
        """Copy this rank's input chunk (complex64, n_local samples) in."""
        self.ctx.bind_stream()
        if x.dtype != torch.complex64 or x.numel() != self.cfg.n_local or not x.is_contiguous():
            raise ValueError("load: contiguous complex64 chunk of n_local samples")
        dst = self.ctx.lib.vsig_chain_input(self.h)
        self.ctx.check(self.ctx.lib.vsig_copy_dev(self.ctx.h, dst, x.data_ptr(), x.numel() * 8), "load")

    def step(self):
        self.ctx.bind_stream()
        rc = self.ctx.lib.vsig_chain_step(self.h)
        if rc:
            raise RuntimeError(f"vsig_chain_step: {rc}: {self.ctx.lib.vsig_chain_last_error(self.h).decode()}")

    def outputs(self):
        """(filtered stream, frame-major spectra) copied into new device tensors."""
        import ctypes as C
        n, nf = C.c_int64(), C.c_int64()
        yp = self.ctx.lib.vsig_chain_filtered(self.h, C.byref(n))
        sp = self.ctx.lib.vsig_chain_spectra(self.h, C.byref(nf))
        y = torch.empty(n.value, dtype=torch.complex64, device=f"cuda:{self.ctx.device}")
        s = torch.empty(nf.value * self.cfg.nfft, dtype=torch.float32, device=y.device)
        self.ctx.check(self.ctx.lib.vsig_copy_dev(self.ctx.h, y.data_ptr(), yp, y.numel() * 8), "y")
        self.ctx.check(self.ctx.lib.vsig_copy_dev(self.ctx.h, s.data_ptr(), sp, s.numel() * 4), "sxx")
        return y, s

    def global_peak(self):
        """(max |c|, global lag, sum |c|, sum |c|^2, n_outputs) of the last step."""
        import ctypes as C
        from ._lib import Peak
        pk, nout = Peak(), C.c_int64()
        rc = self.ctx.lib.vsig_chain_result(self.h, C.byref(pk), C.byref(nout))
        if rc:
            raise RuntimeError(f"vsig_chain_result: {rc}")
        return pk.peak, int(pk.index), pk.sum_abs, pk.sum_abs2, int(nout.value)

    def __del__(self):
        try:
            if self.h:
                self.ctx.lib.vsig_chain_free(self.h)
                self.h = None
        except Exception:
            pass


# ---------------------------------------------------------------------------
# Sharded polyphase channelizer (BASELINE config 4)
# ---------------------------------------------------------------------------
class HipPfbBackend:
    """libvsig.so's PFB kernel on the rank's GPU (product backend)."""

    def __init__(self, proto, nchan: int, device: int):
        from .channelizer import Channelizer
        self.ch = Channelizer(proto, nchan, device)
        self.ctx = self.ch.ctx
        self.dev = torch.device(f"cuda:{device}")

    def empty(self, n, dtype=torch.complex64):
        return torch.zeros(n, dtype=dtype, device=self.dev)

    def pfb_into(self, x, y):
        """frames of x (frame-major, nframes x nchan) into the flat buffer y."""
        C = self.ch.nchan
        nf = self.ch.nframes(int(x.shape[0]))
        self.ch(x, out=y[: nf * C].view(nf, C))


class PfbChain:
    """One rank's part of a time-chunk-sharded C-channel PFB.

    Rank r owns X[r*n, (r+1)*n) and the output frames that start in it
    (frame m reads X[m*C, m*C + ntaps)), so it needs a RIGHT halo of
    ntaps - C samples: the first samples of rank r+1's chunk, received over
    RCCL before the kernel runs.  Concatenating the ranks' frames gives the
    single-stream result exactly ((world*n - ntaps)//C + 1 frames)."""

    def __init__(self, n_local: int, proto, nchan: int, backend, rank: int = 0, world: int = 1,
                 group=None):
        C, ntaps = int(nchan), len(proto)
        if n_local % C:
            raise ValueError("n_local must be a multiple of nchan (frames never straddle ranks)")
        if world > 1 and n_local < ntaps - C:
            raise ValueError("chunk shorter than the PFB halo")
        self.n, self.C, self.ntaps = n_local, C, ntaps
        self.be, self.rank, self.world, self.group = backend, rank, world, group
        self.halo = ntaps - C
        self.rhalo = self.halo if rank < world - 1 else 0
        self.nframes = n_local // C if rank < world - 1 else max(0, (n_local - ntaps) // C + 1)
        self.x_ext = backend.empty(n_local + self.halo)                 # [chunk | right halo]
        self.y = backend.empty(max(self.nframes, 1) * C)                # frame-major

    @property
    def x(self):
        return self.x_ext[: self.n]

    @property
    def frame0(self):
        """Global index of this rank's first frame."""
        return self.rank * (self.n // self.C)

    def step(self):
        r, w, h = self.rank, self.world, self.halo
        if w > 1 and h > 0:
            ops = []
            if r > 0:
                ops.append(dist.P2POp(dist.isend, self.x_ext[:h], r - 1, group=self.group))
            if r < w - 1:
                ops.append(dist.P2POp(dist.irecv, self.x_ext[self.n: self.n + h], r + 1,
                                      group=self.group))
            for req in dist.batch_isend_irecv(ops):
                req.wait()
        if self.nframes > 0:
            self.be.pfb_into(self.x_ext[: self.n + self.rhalo], self.y)

    def frames(self):
        """(nframes, C) view of this rank's output."""
        return self.y[: self.nframes * self.C].view(self.nframes, self.C)
