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

The compute steps go through a backend object and the exchanges through a
transport object, so that the same orchestration runs in production (HipBackend
on libvsig.so, TorchTransport = torch.distributed over RCCL), on CPU under gloo
(tests/test_shard_gloo.py) and as several ranks in one process on one GPU
(HipBackend + NativeTransport over the library's loopback,
tests/test_gpu_shard_threads.py).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch
import torch.distributed as dist

__all__ = ["ChainConfig", "HipBackend", "StreamChain", "combine_peaks", "HipPfbBackend",
           "PfbChain", "NativeChain", "Loopback", "TorchTransport", "NativeTransport"]


@dataclass
class ChainConfig:
    n_local: int                 # input samples per rank
    taps: np.ndarray             # FIR taps (real or complex)
    decim: int = 1
    nfft: int = 8192             # PSD frame = hop (non-overlapping)
    template: np.ndarray | None = None   # sync preamble (None: no xcorr stage)
    window: str = "hann"
    freq_shift: float = 0.0      # apply_frequency_shift before the FIR (fused into its loads),
    sample_rate: float = 1.0     # phase from the global sample index (utils.py:120-127)

    def validate(self, world: int):
        ny = self.n_local // self.decim
        if self.n_local % self.decim:
            raise ValueError("n_local must be a multiple of decim")
        if ny % self.nfft:
            raise ValueError("n_local/decim must be a multiple of nfft (frames never straddle chunks)")
        if self.template is not None and world > 1 and ny < len(self.template) - 1:
            raise ValueError("chunk shorter than the template halo")
        # the left halo is ntaps-1 samples rounded up to 16 (StreamChain.hist:
        # 128-byte-aligned segment starts); a shorter chunk would make the send
        # slice x_ext[n:n+hist] overlap the receive buffer x_ext[:hist] of one
        # sendrecv (chain.hip's vsig_chain_create rejects the same configs)
        if world > 1 and self.n_local < fir_history(len(self.taps)):
            raise ValueError("chunk shorter than the FIR halo "
                             f"(n_local {self.n_local} < {fir_history(len(self.taps))})")


def fir_history(ntaps: int) -> int:
    """Left-halo length of a time chunk: ntaps - 1 input samples rounded up to a
    multiple of 16 (so [halo | chunk]'s FIR segments start on 128-byte lines)."""
    return (ntaps - 1 + 15) // 16 * 16


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


class TorchTransport:
    """Exchanges over torch.distributed (production: backend 'nccl' = RCCL over
    xGMI; gloo on CPU): non-blocking point-to-point halos and an asynchronous
    all-gather, each returning handles for wait()."""

    def __init__(self, group=None):
        self.group = group

    def exchange_start(self, send, dst, recv, src):
        ops = []
        if send is not None and dst is not None:
            ops.append(dist.P2POp(dist.isend, send, dst, group=self.group))
        if recv is not None and src is not None:
            ops.append(dist.P2POp(dist.irecv, recv, src, group=self.group))
        return dist.batch_isend_irecv(ops) if ops else []

    def all_gather_start(self, rows, rec):
        return [dist.all_gather_into_tensor(rows, rec, group=self.group, async_op=True)]

    @staticmethod
    def wait(handles):
        for h in handles or ():
            h.wait()


class NativeTransport:
    """Exchanges through a C vsig_transport (include/vsig.h): the library's
    in-process Loopback (ranks as threads of one process, e.g. several ranks on
    one GPU) or its RCCL transport.  Blocking sendrecv / allgather ordered on
    torch's current stream (the call returns once the partner has the data;
    ctypes releases the GIL around it, so rank threads proceed in parallel)."""

    def __init__(self, t):
        self.t = t

    @staticmethod
    def _ptr_bytes(x):
        return (x.data_ptr(), x.numel() * x.element_size()) if x is not None else (None, 0)

    def exchange_start(self, send, dst, recv, src):
        sp, sb = self._ptr_bytes(send if dst is not None else None)
        rp, rb = self._ptr_bytes(recv if src is not None else None)
        if sp is None and rp is None:
            return []
        st = torch.cuda.current_stream().cuda_stream
        rc = self.t.sendrecv(self.t.user, sp, sb, -1 if sp is None else int(dst), rp, rb,
                             -1 if rp is None else int(src), st)
        if rc:
            raise RuntimeError(f"transport sendrecv failed ({rc})")
        return []

    def all_gather_start(self, rows, rec):
        st = torch.cuda.current_stream().cuda_stream
        rc = self.t.allgather(self.t.user, rec.data_ptr(), rows.data_ptr(),
                              rec.numel() * rec.element_size(), st)
        if rc:
            raise RuntimeError(f"transport allgather failed ({rc})")
        return []

    @staticmethod
    def wait(handles):
        pass


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

    def empty(self, n, dtype=torch.complex64):
        return torch.zeros(n, dtype=dtype, device=self.dev)

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

    def check_refine(self):
        """Raise RefineFault if a refine of this rank faulted since the last
        check (the fault word is sticky on the device; synchronises)."""
        self.dsp.check_refine(self.ctx)

    # -- the refine beside the next step (StreamChain overlap_refine) ---------
    def set_overlap_refine(self, on: bool):
        """The context's "refine_async" option (vsig.h): the correlator's exact
        refine runs on the context's refine stream, behind an event."""
        self.ctx.check(self.ctx.lib.vsig_set_option(self.ctx.h, b"refine_async", int(bool(on))),
                       "refine_async")

    def refine_stream(self):
        """The stream the refine runs on, as a torch stream (its consumers --
        the peak records' all-gather -- are issued there)."""
        return torch.cuda.ExternalStream(self.ctx.lib.vsig_refine_stream(self.ctx.h), device=self.dev)

    def join_refine(self):
        """torch's current stream waits for the last refine (an event)."""
        self.ctx.bind_stream()
        self.ctx.check(self.ctx.lib.vsig_refine_join(self.ctx.h), "refine_join")


class StreamChain:
    """One rank's part of the sharded chain (world = 1: the plain chain)."""

    def __init__(self, cfg: ChainConfig, backend, rank: int = 0, world: int = 1, group=None,
                 transport=None, overlap_refine: bool = False):
        """overlap_refine: the correlator's exact-argmax refine of step k runs on
        the backend's refine stream beside step k + 1's FIR (which writes the
        other of two filtered-stream buffers, the refine re-reading this one);
        the peak records' all-gather is issued on that stream and global_peak
        joins it.  Needs a backend with set_overlap_refine (HipBackend); costs
        a second filtered-stream buffer (4.3 GB at config 5)."""
        cfg.validate(world)
        self.cfg, self.be, self.rank, self.world, self.group = cfg, backend, rank, world, group
        self.tr = transport if transport is not None else TorchTransport(group)
        # the left halo: ntaps - 1 samples, rounded up to a multiple of 16 so
        # that [halo | chunk] puts the FIR's segment starts on 128-byte lines
        # (D = 4: lo2 = 256 at 255 taps; the surplus samples are never read by
        # a tap; profiles/r05_fir_align_ab.txt)
        self.hist = fir_history(len(cfg.taps))
        self.ny = cfg.n_local // cfg.decim
        self.L = len(cfg.template) if cfg.template is not None else 0
        self.yhalo = (self.L - 1) if (self.L and rank < world - 1) else 0
        self.x_ext = backend.empty(self.hist + cfg.n_local)          # [left halo | chunk]
        self.overlap = bool(overlap_refine and self.L and hasattr(backend, "set_overlap_refine"))
        if self.overlap:
            backend.set_overlap_refine(True)
        # [chunk out | right halo]; two of them with overlap_refine (step k uses
        # buffer k mod 2, see _begin_step)
        self._y_bufs = [backend.empty(self.ny + max(self.L - 1, 0))
                        for _ in range(2 if overlap_refine and self.L else 1)]
        self.sxx = backend.empty((self.ny // cfg.nfft) * cfg.nfft, torch.float32)
        # peak records, double-buffered: the all-gather of step k runs behind
        # step k + 1 (it is waited for only before step k + 2 reuses its slot,
        # or by global_peak); every rank's records land in place (no copies)
        self._recs = backend.empty(2 * 4, torch.float64).view(2, 4)
        self._rows = backend.empty(2 * 4 * world, torch.float64).view(2, world * 4)
        self._gather = [None, None]
        self._slot = 1
        self.y_ext = self._y_bufs[self._slot % len(self._y_bufs)]
        self.peak_rows = None
        self._wt = None                   # exposed-wait events (enable_wait_timing)

    @property
    def x(self):
        """The rank's own input chunk (fill it before step())."""
        return self.x_ext[self.hist:]

    @property
    def y(self):
        return self.y_ext[: self.ny]

    @property
    def rec(self):
        """This step's peak record."""
        return self._recs[self._slot]

    # -- per-rank diagnostics (bench.py at world > 1) --------------------------
    def enable_wait_timing(self, on: bool = True):
        """Bracket the step's three exposed waits with timing events on the
        launch stream: the all-gather slot wait at the step start ('gather'),
        the left-halo wait before the FIR's first outputs ('left_halo') and
        the right-halo wait before the correlator ('right_halo').  The first
        event completes when the stream's previous work has, the second when
        the wait is satisfied, so their difference is the GPU time the stream
        stalls on the exchange -- measured, not inferred.  Off (None) by
        default; reset by each call."""
        self._wt = {"gather": [], "left_halo": [], "right_halo": []} if on else None

    def _waited(self, name, wait, *a):
        if self._wt is None:
            return wait(*a)
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        r = wait(*a)
        e1.record()
        self._wt[name].append((e0, e1))
        return r

    def wait_ms(self, steps: int | None = None):
        """{wait: mean exposed ms per step} of the recorded steps (waits that a
        rank does not have, e.g. rank 0's left halo, count as 0); synchronises."""
        out = {}
        for k, evs in (self._wt or {}).items():
            if evs:
                evs[-1][1].synchronize()
            tot = sum(a.elapsed_time(b) for a, b in evs)
            out[k] = tot / steps if steps else (tot / len(evs) if evs else 0.0)
        return out

    def _begin_step(self):
        self._slot ^= 1
        self.y_ext = self._y_bufs[self._slot % len(self._y_bufs)]
        work, self._gather[self._slot] = self._gather[self._slot], None
        if work:
            self._waited("gather", self.tr.wait, work)   # the all-gather two steps back

    def _gather_peaks(self):
        rows = self._rows[self._slot]
        if self.overlap:          # behind the refine, not in front of the next FIR
            with torch.cuda.stream(self.be.refine_stream()):
                self._gather[self._slot] = self.tr.all_gather_start(rows, self.rec)
        else:
            self._gather[self._slot] = self.tr.all_gather_start(rows, self.rec)
        return list(rows.view(self.world, 4).unbind(0))

    def _exchange_start(self, send, dst, recv, src):
        return self.tr.exchange_start(send, dst, recv, src)

    def _exchange_wait(self, reqs):
        self.tr.wait(reqs)

    def _exchange(self, send, dst, recv, src):
        self._exchange_wait(self._exchange_start(send, dst, recv, src))

    def _fir(self, be, a, b, y):
        """FIR of the rank's input samples [a, b) (plus their history) into y."""
        x = self.x_ext[a: b + self.hist]
        if self.cfg.freq_shift:
            be.fir_into(x, self.hist, y, self.rank * self.cfg.n_local - self.hist + a)
        else:
            be.fir_into(x, self.hist, y)

    def _fir_first(self, be):
        """FIR of the chunk with the left-halo exchange hidden behind it:
        outputs from a decimation-aligned s >= ntaps-1 on need only the rank's
        own samples and are filtered while the halo is in flight; the first
        s outputs follow once it has landed."""
        r, w, hist, n = self.rank, self.world, self.hist, self.cfg.n_local
        D = self.cfg.decim

        def run(a, b):
            self._fir(be, a, b, self.y_ext[a // D: b // D])
        if not (w > 1 and hist > 0):
            run(0, n)
            return
        reqs = self._exchange_start(self.x_ext[n: n + hist] if r < w - 1 else None,
                                    r + 1 if r < w - 1 else None,
                                    self.x_ext[: hist] if r > 0 else None,
                                    r - 1 if r > 0 else None)
        s = -(-hist // D) * D
        if s < n:
            run(s, n)
        self._waited("left_halo", self._exchange_wait, reqs)
        run(0, min(s, n))

    def step(self):
        """One step, every stage on the current stream: FIR (left halo hidden
        behind its bulk), the right-halo exchange started behind it, the PSD
        while the halo is in flight, then the correlator once it has landed,
        then the peak records' all-gather (asynchronous, see __init__).
        (Three-stream and sub-chunked pipelines measured slower on MI355X:
        DESIGN.md section 5; so did the PSD after the correlator, +0.7-1.3 %:
        the stage right after the FIR runs at the lowest clock, and the
        correlator pays more for it than the PSD, profiles/r06_stage_order_ab.txt.)"""
        self._begin_step()
        r, w, ny, L = self.rank, self.world, self.ny, self.L
        be = self.be
        self._fir_first(be)
        reqs = []
        if w > 1 and L > 1:
            reqs = self._exchange_start(self.y_ext[: L - 1] if r > 0 else None,
                                        r - 1 if r > 0 else None,
                                        self.y_ext[ny: ny + L - 1] if r < w - 1 else None,
                                        r + 1 if r < w - 1 else None)
        be.psd_into(self.y_ext[: ny], self.sxx)
        if reqs or (w > 1 and L > 1):
            self._waited("right_halo", self._exchange_wait, reqs)
        if L:
            halo = (L - 1) if r < w - 1 else 0
            be.xcorr_peak(self.y_ext[: ny + halo], self.rec)
            self.peak_rows = self._gather_peaks() if w > 1 else [self.rec]

    def global_peak(self):
        """(max |c|, global lag, sum |c|, sum |c|^2, n_outputs) of the last step.
        A refine fault -- on this rank since the last call (the backend's
        sticky fault word) or on any rank (its gathered row's poisoned index,
        refine.hip poison_record) -- raises RefineFault."""
        if self.overlap:
            self.be.join_refine()
        self.tr.wait(self._gather[self._slot])
        check = getattr(self.be, "check_refine", None)
        if check is not None:
            check()
        rows = []
        for r, t in enumerate(self.peak_rows):
            h = t.detach().cpu().reshape(4)
            idx = int(h.view(torch.int64)[1].item())
            if idx < 0:
                from ._lib import RefineFault
                raise RefineFault(f"exact-argmax refine faulted on rank {r} (poisoned peak record)")
            rows.append((float(h[0]), r * self.ny + idx, float(h[2]), float(h[3])))
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
        t._owner = self          # t.user points into this loopback: keep it alive with t
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
            msg = self.ctx.lib.vsig_chain_last_error(self.h).decode()
            if rc == -6:                   # VSIG_E_REFINE: the exact-argmax contract broke
                from ._lib import RefineFault
                raise RefineFault(f"vsig_chain_result: {msg}")
            raise RuntimeError(f"vsig_chain_result: {rc}: {msg}")
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
                 group=None, transport=None):
        C, ntaps = int(nchan), len(proto)
        if n_local % C:
            raise ValueError("n_local must be a multiple of nchan (frames never straddle ranks)")
        if world > 1 and n_local < ntaps - C:
            raise ValueError("chunk shorter than the PFB halo")
        self.n, self.C, self.ntaps = n_local, C, ntaps
        self.be, self.rank, self.world, self.group = backend, rank, world, group
        self.tr = transport if transport is not None else TorchTransport(group)
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
            self.tr.wait(self.tr.exchange_start(self.x_ext[:h] if r > 0 else None,
                                                r - 1 if r > 0 else None,
                                                self.x_ext[self.n: self.n + h] if r < w - 1 else None,
                                                r + 1 if r < w - 1 else None))
        if self.nframes > 0:
            self.be.pfb_into(self.x_ext[: self.n + self.rhalo], self.y)

    def frames(self):
        """(nframes, C) view of this rank's output."""
        return self.y[: self.nframes * self.C].view(self.nframes, self.C)
