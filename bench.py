"""Benchmark: Msamples/s of complex64 IQ through the FIR -> decimate -> FFT-PSD
-> xcorr-sync chain on 1..N MI355X GPUs, with the dominant kernel's achieved
HBM bandwidth against the roofline and the CPU reference path beside it.

Default workload = BASELINE configs[4] (config 5, the metric's full chain):
one synthetic capture of 2**31 complex64 samples (2 GS/s for 1.07 s), 255-tap
FIR, decimate by 4, 8192-point Hann PSD (hop 8192) of the decimated stream,
4096-sample template valid correlation of the decimated stream with the fused
|c| argmax (+ its exact refine).  Time-chunk partition: N GPUs own 2**31 / N
contiguous samples each (strong scaling), exchanging only the FIR / correlation
halos and 32-byte peak records over RCCL.

  python bench.py [--gpus N --steps K --warmup W]   # N > 1: starts its N ranks itself
  python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...
  python bench.py --workload c2       # configs[1]: 2**28 samples / GPU, D = 1 (+ the sync
                                      #   stage), north_star's FIR+FFT >= 70 % HBM target
  python bench.py --workload sync     # configs[2]: 4096-sample preamble over 2**30
  python bench.py --workload pfb      # configs[3]: 64-channel PFB, 2**29 samples / GPU
  python bench.py --freq-shift 3e8    # the chain with the NCO mixer fused into the FIR

Inputs are generated on the device before timing (data resident in HBM).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Msamples/s c64 through FIR+FFT+xcorr chain; 1/2/4/8 GPU + %HBM roofline"
HBM_PEAK_GBS = 8000.0          # MI355X spec (MI355X_MICROARCH.md: 8.0 TB/s)
FP32_PEAK_TF = 157.3           # MI355X FP32 vector peak (packed FMA), MI355X_MICROARCH.md
TONES = ((1.0, 0.05), (0.5, 0.11), (0.25, -0.20))


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def design(ntaps, L, decim=1):
    import scipy.signal
    taps = scipy.signal.firwin(ntaps, 0.2).astype(np.float32)
    rng = np.random.default_rng(4096)
    b = rng.integers(0, 2, size=(2, L * decim))
    pre = (((2 * b[0] - 1) + 1j * (2 * b[1] - 1)) / np.sqrt(2)).astype(np.complex64)
    # The template is the preamble as it leaves the receive filter and the
    # decimator (causal part, every decim-th sample): the filtered, decimated
    # capture contains it exactly at the planted offset / decim.
    tmpl = np.convolve(pre, taps)[:L * decim][::decim].astype(np.complex64)
    return taps, pre, tmpl


def generate_chunk(x: torch.Tensor, g0: int, seed: int, pre: np.ndarray, k0: int):
    """x[i] = sum_t A_t exp(j 2 pi f_t (g0 + i)) + CN(0,1) noise (+ preamble at
    global sample k0), written in place on the device, in 2**24-sample slabs."""
    n = x.shape[0]
    gen = torch.Generator(device=x.device)
    gen.manual_seed(seed)
    slab = 1 << 24
    for s in range(0, n, slab):
        m = min(slab, n - s)
        idx = torch.arange(g0 + s, g0 + s + m, device=x.device, dtype=torch.float64)
        acc = torch.randn(m, dtype=torch.complex64, device=x.device, generator=gen)
        for a, f in TONES:
            ph = torch.remainder(idx * f, 1.0) * (2 * np.pi)
            acc += (a * torch.polar(torch.ones_like(ph), ph)).to(torch.complex64)
        x[s:s + m] = acc
    lo, hi = max(k0, g0), min(k0 + len(pre), g0 + n)
    if lo < hi:
        x[lo - g0:hi - g0] += torch.from_numpy(pre[lo - k0:hi - k0]).to(x.device)


def cpu_baseline(samples, taps, nfft, tmpl, decim=1):
    """The reference's CPU path (oracle: np.convolve / scipy.signal.spectrogram /
    np.correlate, single-threaded numpy) timed on a bounded sample."""
    from oracle import ref
    x = ref.synth_iq(samples, seed=99)
    t0 = time.perf_counter()
    y = ref.fir_filter(x, taps, decim)
    ref.spectrum(y, 1.0, "hann", nfft, 0, nfft)
    c, lags = ref.cross_correlate_signals(tmpl, y, "valid")
    ref.find_correlation_peak(c, lags)
    dt = time.perf_counter() - t0
    return dict(value=round(samples / dt / 1e6, 3), unit="Msamples/s", cores=1, kind="port",
                sample=(f"{samples} samples (2**{int(np.log2(samples))}) of the same chain: "
                        f"np.convolve {len(taps)} taps + [::{decim}], scipy spectrogram nfft={nfft}, "
                        f"np.correlate complex128 L={len(tmpl)} valid + find_correlation_peak; "
                        f"{dt:.2f} s, 1 thread"),
                seconds=round(dt, 3))


def cpu_allowance():
    """(cores this process may use, how that was determined): the affinity
    mask, capped by a cgroup CPU quota (v2 cpu.max, v1 cfs_quota_us) where one
    is set; OMP_NUM_THREADS (the pool sets it to the box's CPU share) is
    recorded and caps it too."""
    aff = len(os.sched_getaffinity(0))
    n, src = aff, [f"sched_getaffinity={aff}"]
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    if quota is not None:
        src.append(f"cgroup quota {quota:g} cores")
        n = min(n, max(1, int(quota)))
    else:
        src.append("no cgroup quota")
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        src.append(f"OMP_NUM_THREADS={omp}")
        n = min(n, int(omp))
    return n, ", ".join(src)


def cpu_baseline_allcores(samples, taps, nfft, tmpl, workers, decim=1):
    """The same CPU chain as cpu_baseline on `workers` processes, one time
    chunk each with its halos (SURVEY.md §8(d)'s all-cores variant); value =
    all chunks' samples / the wall time of the parallel map (worker start-up
    and imports excluded by a warm-up map)."""
    import multiprocessing as mp
    from oracle import ref
    ctx = mp.get_context("spawn")       # fresh interpreters: no GPU state in the workers
    jobs = [(samples, 1000 + w, taps, nfft, tmpl, decim) for w in range(workers)]
    with ctx.Pool(workers) as pool:
        pool.map(ref.chain_chunk_seconds, [(1 << 15, w, taps, nfft, tmpl, decim)
                                           for w in range(workers)])
        t0 = time.perf_counter()
        secs = pool.map(ref.chain_chunk_seconds, jobs)
        dt = time.perf_counter() - t0
    return dict(value=round(workers * samples / dt / 1e6, 3), unit="Msamples/s", cores=workers,
                kind="port",
                sample=(f"{workers} processes x {samples} samples (2**{int(np.log2(samples))}) of "
                        f"the chain with halos, {dt:.2f} s wall (per-chunk {min(secs):.2f}-"
                        f"{max(secs):.2f} s)"),
                seconds=round(dt, 3))


def xcorr_block(L):
    """Overlap-save block size the correlator plans for a template of L
    (vsig_api.hip os_size_xcorr)."""
    return 4096 if L <= 1024 else 8192 if L <= 2048 else 16384


def practical_ceiling(kind):
    """The best rate the pool's boxes reached on an access pattern like the
    kernel's (tools/membw.py probes, the newest profiles/r0N_membw.json):
    'read4to1' for the decimating FIR's 8 B read : 2 B written per sample
    (every lane width / unroll / non-temporal variant of it), 'copy' (unrolled
    lanes, loads in flight, NT hints) for the 1:1 streams.  (GB/s, source)"""
    for name in ("r05_membw.json", "r02_membw.json"):
        try:
            d = json.load(open(os.path.join(ROOT, "profiles", name)))
        except Exception:
            continue
        prefs = ("read4to1", "r4w") if kind == "read4to1" else ("probe_u",)
        vals = [v[1] for k, v in d.items() if k.startswith(prefs) and isinstance(v, list)]
        if vals:
            return max(vals), f"profiles/{name} max({'|'.join(p + '*' for p in prefs)})"
    return None


def load_traffic(key):
    """Measured HBM bytes per launch from a committed rocprofv3 --pmc summary
    (profiles/pmc_*.json, corrected as MI355X_MICROARCH.md §HBM prescribes)."""
    import glob
    import re

    def order(p):       # newest profile round / version last (r02_v14 after r02_v8)
        m = re.search(r"_r(\d+)_v(\d+)", os.path.basename(p))
        return (int(m.group(1)), int(m.group(2))) if m else (0, 0)
    best = None
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_*.json")), key=order):
        try:
            d = json.load(open(p))
        except Exception:
            continue
        if d.get("config_key") == key:
            best = d
    return best


WORKLOADS = {
    # name: (decim, samples, per_gpu (weak) or total (strong), label)
    "c5": (4, 1 << 31, False, "BASELINE configs[4]: full chain FIR -> decimate 4 -> FFT PSD -> "
                              "xcorr over a 2**31-sample capture, time-chunk partition"),
    "c2": (1, 1 << 28, True, "BASELINE configs[1] chain + sync: 2**28 samples per GPU, D = 1"),
}


def rehearsal_env(rank: int) -> dict:
    """--rehearse-one-gpu: every rank on cuda:0 of a one-GPU box (the pool's),
    over the production RCCL path.  RCCL refuses two ranks on one device of one
    host, so each rank names its own host (NCCL_HOSTID) and the ranks talk over
    RCCL's socket transport on loopback (P2P / SHM off).  Exercises every RCCL
    call, stream dependency and the per-rank line of an N-GPU run; its times are
    N ranks sharing one GPU and sockets for xGMI -- not a scaling measurement
    (tests/test_gpu_rccl.py, tests/test_gpu_bench.py)."""
    return {"NCCL_HOSTID": f"vsig-rank{rank}", "NCCL_SOCKET_IFNAME": "lo", "NCCL_NET": "Socket",
            "NCCL_P2P_DISABLE": "1", "NCCL_SHM_DISABLE": "1", "LOCAL_RANK": "0"}


def launch_ranks(n: int, argv: list[str]) -> int:
    """`bench.py --gpus N` without a launcher: start N child processes of this
    script (one per GPU, RANK = LOCAL_RANK = r, WORLD_SIZE = N, rendezvous on
    127.0.0.1) -- before anything here touches the GPU, and as children, never
    by exec.  The parent holds the rendezvous store itself (bound to a free port
    before any child starts, as torchrun's agent does: the children connect as
    clients, so no port can be taken in between).  Rank 0's stdout carries the
    one JSON line.  Returns the first non-zero child exit code (the others are
    stopped then), else 0; on SIGTERM / Ctrl-C the children are stopped too."""
    import signal
    import subprocess
    from torch.distributed import TCPStore
    store = TCPStore("127.0.0.1", 0, world_size=None, is_master=True, wait_for_workers=False)
    port = str(store.port)
    procs = []

    def _term(signum, frame):
        raise SystemExit(128 + signum)
    old = signal.signal(signal.SIGTERM, _term)
    rc = 0
    try:
        rehearse = "--rehearse-one-gpu" in argv
        for r in range(n):
            env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                       LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=port,
                       TORCHELASTIC_USE_AGENT_STORE="True", TORCHELASTIC_RESTART_COUNT="0")
            if rehearse:
                env.update(rehearsal_env(r))
            procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv],
                                          env=env))
        live = list(procs)
        while live:
            for p in list(live):
                code = p.poll()
                if code is None:
                    continue
                live.remove(p)
                if code != 0 and rc == 0:
                    rc = code if code > 0 else 1
                    log(f"bench: rank {procs.index(p)} exited with {code}; stopping the others")
                    for q in live:
                        q.terminate()
            time.sleep(0.05)
    finally:
        signal.signal(signal.SIGTERM, old)
        for p in procs:                   # nothing outlives the launcher
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=15)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
        del store
    return rc


def _launcher_selftest(args, world, rank, local):
    """Rendezvous over gloo (CPU only) and report what each rank was given
    (tests/test_bench_launch.py)."""
    dist.init_process_group("gloo")
    info = {k: os.environ.get(k) for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR",
                                           "MASTER_PORT")}
    info["pid"] = os.getpid()
    json.dump(info, open(os.path.join(args.launcher_selftest, f"rank{rank}.json"), "w"))
    if os.environ.get("VSIG_SELFTEST_HANG"):     # the launcher's cleanup test: stay alive
        time.sleep(120)
    t = torch.tensor([rank + 1.0])
    dist.all_reduce(t)
    # the per-rank diagnostics' gather and summary, on made-up numbers (rank r's
    # stages r + 1 ms, its right-halo wait 0.1 r ms; the last rank the slowest)
    row = rank_row(1e-3 * (10 + rank) * 5, 5, {"fir": 1.0 + rank, "psd": 0.5, "xcorr": 2.0},
                   {"right_halo": 0.1 * rank, "gather": 0.01})
    ranks = summarize_ranks(gather_rank_rows(row, world, torch.device("cpu")))
    if rank == 0:
        print(json.dumps({"metric": METRIC, "n_gpus": world, "rccl_world": dist.get_world_size(),
                          "sum_ranks": float(t.item()), "ranks": ranks}), flush=True)
    dist.destroy_process_group()


# Per-rank diagnostics at world > 1: each rank's own
# elapsed time, its stage means (HIP events, vsig_timing) and the exposed
# waits of its exchanges (StreamChain.enable_wait_timing), all-gathered.
RANK_FIELDS = ("ms_per_step", "fir", "psd", "xcorr", "refine", "left_halo_wait",
               "right_halo_wait", "gather_wait", "fir_ghz", "psd_ghz", "xcorr_ghz")
CLOCK_STAGES = ("fir", "psd", "xcorr")


def rank_row(elapsed, steps, stages, waits, clocks=None):
    """One rank's diagnostics in ms (per step; a stage or wait it lacks is 0)
    and its stages' effective clocks in GHz (0 if not measured)."""
    row = {"ms_per_step": elapsed / steps * 1e3}
    for k in ("fir", "psd", "xcorr", "refine"):
        row[k] = float(stages.get(k, 0.0))
    if "refine_overlapped_span" in stages:     # the refine beside the next step's FIR
        row["refine"] = float(stages["refine_overlapped_span"])
    for k in ("left_halo", "right_halo", "gather"):
        row[k + "_wait"] = float(waits.get(k, 0.0))
    for k in CLOCK_STAGES:
        row[k + "_ghz"] = float((clocks or {}).get(k, 0.0))
    return row


def stage_clocks(lib, h, run, nsteps):
    """Effective clock of each stage (GHz) over `nsteps` untimed steps `run()`
    with the library's clock sinks on (vsig_clock_*: the shader clock against
    the 100 MHz real-time counter over every 64th block's lifetime)."""
    import ctypes as C
    if lib.vsig_clock_enable(h, 1) != 0:
        return {}
    for _ in range(nsteps):
        run()
    torch.cuda.synchronize()
    out = {}
    for name in CLOCK_STAGES + ("pfb",):
        ghz, ticks = C.c_double(), C.c_int64()
        if lib.vsig_clock_read(h, name.encode(), C.byref(ghz), C.byref(ticks)) == 0 and ticks.value:
            out[name] = round(ghz.value, 3)
    lib.vsig_clock_enable(h, 0)
    return out


def gather_rank_rows(row, world, dev):
    """All ranks' rows on every rank (a float64 all-gather: RCCL on the GPU,
    gloo on the CPU)."""
    mine = torch.tensor([row[k] for k in RANK_FIELDS], dtype=torch.float64, device=dev)
    out = torch.empty(world * len(RANK_FIELDS), dtype=torch.float64, device=dev)
    dist.all_gather_into_tensor(out, mine)
    vals = out.cpu().view(world, len(RANK_FIELDS)).tolist()
    return [dict(zip(RANK_FIELDS, v)) for v in vals]


def summarize_ranks(rows):
    """min / max (and the rank holding the max) of every field over the ranks,
    the rank that set ms_per_step (the max over ranks), and the rows."""
    out = {"world": len(rows)}
    for k in RANK_FIELDS:
        v = [r[k] for r in rows]
        i = int(np.argmax(v))
        out[k] = {"min": round(min(v), 4), "max": round(v[i], 4), "max_rank": i}
    out["pace_rank"] = out["ms_per_step"]["max_rank"]
    out["per_rank"] = [{k: round(r[k], 4) for k in RANK_FIELDS} for r in rows]
    return out


def run_chain_leg(args, n, decim, rank, world, local, dev, steps, warmup):
    """Build the chain for n input samples per rank at decimation `decim`, fill
    it on the device, run `warmup` untimed and `steps` timed steps (barrier +
    synchronize on both sides, max over ranks) and return the elapsed time,
    the per-stage HIP-event means and every stage against its roof."""
    from vector_amd.shard import ChainConfig, HipBackend, StreamChain
    from vector_amd._lib import get_context
    granule = args.nfft * decim
    if n % granule:
        raise SystemExit(f"samples per GPU ({n}) must be a multiple of nfft * decim ({granule})")
    taps, pre, tmpl = design(args.ntaps, args.template, decim)
    ctx0 = get_context(local)
    if args.no_refine:
        ctx0.check(ctx0.lib.vsig_set_option(ctx0.h, b"refine", 0), "refine")
    cfg = ChainConfig(n_local=n, taps=taps, decim=decim, nfft=args.nfft, template=tmpl,
                      freq_shift=args.freq_shift, sample_rate=args.sample_rate)
    be = HipBackend(cfg, local)
    # the exact-argmax refine of step k beside step k + 1's FIR (its own stream,
    # a second filtered-stream buffer; shard.StreamChain overlap_refine)
    chain = StreamChain(cfg, be, rank, world, overlap_refine=not args.no_overlap_refine)
    N = world * n
    ny_total = N // decim
    k0 = (ny_total // 2 + 12_345) * decim     # global input sample of the preamble
    if args.freq_shift:   # plant the preamble so that it leaves the mixer unrotated
        ph = 2 * np.pi * args.freq_shift * ((k0 + np.arange(len(pre))) / args.sample_rate)
        pre = (pre * np.exp(-1j * ph)).astype(np.complex64)
    generate_chunk(chain.x, rank * n, 20250718 + rank, pre, k0)
    torch.cuda.synchronize()

    def barrier():
        if world > 1:
            dist.barrier()

    for _ in range(warmup):
        chain.step()
    torch.cuda.synchronize()
    barrier()
    lib, h = be.ctx.lib, be.ctx.h
    lib.vsig_timing_reset(h)
    lib.vsig_timing_enable(h, 0 if args.no_kernel_timing else 1)
    torch.cuda.synchronize()
    barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        chain.step()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    barrier()
    lib.vsig_timing_enable(h, 0)
    elapsed = t1 - t0

    # per-kernel durations from HIP events on the launch stream
    import ctypes as C
    stages = {}
    for name in ("fir", "psd", "xcorr", "refine"):
        tot, cnt = C.c_double(), C.c_int64()
        lib.vsig_timing_read(h, name.encode(), C.byref(tot), C.byref(cnt))
        if cnt.value:
            stages[name] = tot.value / cnt.value
    if chain.overlap and "refine" in stages:
        # beside the next step's FIR the refine's blocks start as FIR waves free
        # a SIMD's registers, so its span is the FIR's; what the step pays for it
        # is not this span (ms_per_step against --no-overlap-refine)
        stages["refine_overlapped_span"] = stages.pop("refine")
    # untimed diagnostic steps after the timed loop (the timed steps stay the
    # single-rank path's): each stage's effective clock, and at world > 1 the
    # exposed waits of the exchanges
    clocks, waits = {}, {}
    ndiag = 0 if args.no_kernel_timing else 3
    if ndiag:
        clocks = stage_clocks(lib, h, chain.step, ndiag)
        if world > 1:
            chain.enable_wait_timing(True)
            for _ in range(ndiag):
                chain.step()
            torch.cuda.synchronize()
            waits = chain.wait_ms(ndiag)
            chain.enable_wait_timing(False)
        barrier()
    ranks = None
    if world > 1:
        # every rank's own elapsed time, stage means, clocks and exposed waits,
        # gathered so the line says which rank and which exchange set the pace
        rows = gather_rank_rows(rank_row(elapsed, steps, stages, waits, clocks), world, dev)
        ranks = summarize_ranks(rows)
        elapsed = max(r["ms_per_step"] for r in rows) * steps * 1e-3
    ny = n // decim
    bytes_per_launch = {"fir": 8 * n + 8 * ny, "psd": 8 * ny + 4 * ny,
                        "xcorr": 8 * (ny + chain.yhalo)}
    m, lag, s1, s2, nout = chain.global_peak()
    check = {"sync_lag": lag, "expected": k0 // decim, "ok": bool(lag == k0 // decim)}
    ms_per_step = elapsed / steps * 1e3
    yhalo = chain.yhalo
    overlapped = chain.overlap
    del chain, be
    torch.cuda.empty_cache()

    roof = None
    kstages = {k: v for k, v in stages.items() if k in bytes_per_launch}
    if kstages:
        dom = max(kstages, key=lambda k: kstages[k])
        achieved = bytes_per_launch[dom] / (kstages[dom] * 1e-3) / 1e9
        key = f"{dom}:n={n}:ntaps={args.ntaps}:decim={decim}:nfft={args.nfft}:L={args.template}"
        pmc = load_traffic(key)
        roof = {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": pmc["hbm_bytes_per_launch"] if pmc else None,
                "algorithmic_bytes": bytes_per_launch[dom],
                "avg_launch_ms": round(kstages[dom], 4),
                "traffic_source": pmc["source"] if pmc else None}
        if pmc and "valu_issue_frac" in pmc:
            roof["valu_issue_frac"] = pmc["valu_issue_frac"]
        # the same rate against what a pure stream of this shape reached on the
        # pool's boxes (secondary: the headline frac is against the 8 TB/s spec)
        pc = practical_ceiling("read4to1" if (dom == "fir" and decim == 4) else "copy")
        if pc:
            roof["practical_peak"] = pc[0]
            roof["practical_frac"] = round(achieved / pc[0], 4)
            roof["practical_source"] = pc[1]
    # every stage against its own roof: HBM bytes for all three, and for the
    # correlator (not HBM-bound) the FP32 vector roof with the standard
    # 5 N log2 N FFT flop count (2 FFTs + the spectrum multiply per block)
    stage_roof = {}
    for k, ms in kstages.items():
        gbs = bytes_per_launch[k] / (ms * 1e-3) / 1e9
        stage_roof[k] = {"ms": round(ms, 4), "bytes": bytes_per_launch[k], "GBs": round(gbs, 1),
                         "hbm_frac": round(gbs / HBM_PEAK_GBS, 4)}
        pk = load_traffic(f"{k}:n={n}:ntaps={args.ntaps}:decim={decim}:nfft={args.nfft}:"
                          f"L={args.template}")
        if pk:
            stage_roof[k]["traffic"] = pk["hbm_bytes_per_launch"]
            stage_roof[k]["traffic_source"] = pk["source"]
            if "valu_issue_frac" in pk:
                stage_roof[k]["valu_issue_frac"] = pk["valu_issue_frac"]
    if "xcorr" in stages:
        M = xcorr_block(args.template)
        L = args.template
        hop = M - L + 1
        if M == 16384 and hop > 1:      # the API's even hop (16-byte segment loads)
            hop &= ~1
        nb = -(-(ny + yhalo - L + 1) // hop)
        flops = nb * (2 * 5 * M * np.log2(M) + 6 * M)
        tf = flops / (stages["xcorr"] * 1e-3) / 1e12
        stage_roof["xcorr"].update({"flops": int(flops), "TFLOPs": round(tf, 2),
                                    "valu_peak_TFLOPs": FP32_PEAK_TF,
                                    "valu_frac": round(tf / FP32_PEAK_TF, 4), "M": M})
    if "refine" in stages or "refine_overlapped_span" in stages:
        # overlapped: the refine runs beside the next step's FIR (its span there
        # is the FIR's); the step's time beyond its three stages is what stays
        # exposed of it, with the launch gaps between the stages
        stage_roof["refine"] = {"overlapped": overlapped,
                                "ms" if not overlapped else "span_beside_next_fir_ms":
                                    round(stages.get("refine", stages.get("refine_overlapped_span", 0.0)), 4),
                                "step_minus_stages_ms": round(
                                    ms_per_step - sum(stages.get(k, 0.0) for k in ("fir", "psd", "xcorr",
                                                                                    "refine")), 4)}
    # north_star's FIR+FFT target on SURVEY.md §8(d)'s unfused byte count
    # (filter() writes y, spectrum() reads it): 8 + 8/D + 12/D B/sample
    if "fir" in stages and "psd" in stages:
        fp_ms = stages["fir"] + stages["psd"]
        b = bytes_per_launch["fir"] + bytes_per_launch["psd"]
        t = fp_ms * 1e-3
        stage_roof["fir+psd"] = {"ms": round(fp_ms, 4), "GBs": round(b / t / 1e9, 1),
                                 "hbm_frac": round(b / t / 1e9 / HBM_PEAK_GBS, 4),
                                 "bytes_basis": f"{b / n:.0f} B/sample (FIR 8 + 8/D, PSD 12/D)"}
    # the whole step against the chain's algorithmic bytes (SURVEY.md §8(d):
    # 28 B/sample at D = 1 plus the correlator's 8, 15 B/sample at D = 4)
    chain_bytes = sum(bytes_per_launch.values())
    stage_roof["chain"] = {"ms": round(ms_per_step, 4), "bytes_per_gpu": chain_bytes,
                           "GBs_per_gpu": round(chain_bytes / (ms_per_step * 1e-3) / 1e9, 1),
                           "hbm_frac": round(chain_bytes / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                           "bytes_basis": f"{chain_bytes / n:.2f} B/input sample"}
    for k, g in clocks.items():
        if k in stage_roof:
            stage_roof[k]["ghz"] = g
    return {"elapsed": elapsed, "stages": stages, "stage_roof": stage_roof, "roof": roof,
            "check": check, "taps": taps, "tmpl": tmpl, "ranks": ranks, "clocks": clocks}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", choices=("c5", "c2", "pfb", "sync"), default="c5",
                    help="c5: the metric's full chain (default); c2: 2**28/GPU, D=1; "
                         "sync: config 3 preamble correlation over 2**30 samples; pfb: config 4")
    ap.add_argument("--samples", type=int, default=None,
                    help="input samples per GPU (default: the workload's)")
    ap.add_argument("--ntaps", type=int, default=255)
    ap.add_argument("--decim", type=int, default=None, help="(default: the workload's)")
    ap.add_argument("--nfft", type=int, default=8192)
    ap.add_argument("--template", type=int, default=4096)
    ap.add_argument("--cpu-samples", type=int, default=None,
                    help="CPU-baseline sample (default: ~10-15 s of single-core work: "
                         "2**26 samples for the chains, 2**24 for sync, 2**27 for pfb)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-workers", type=int, default=None,
                    help="processes for the all-cores CPU baseline (default: this process's CPU "
                         "allowance, bench.cpu_allowance, within host memory)")
    ap.add_argument("--no-kernel-timing", action="store_true")
    ap.add_argument("--no-overlap-refine", action="store_true",
                    help="run the refine on the step's stream (not beside the next step's FIR)")
    ap.add_argument("--no-refine", action="store_true",
                    help="skip the correlator's exact-argmax refine pass (A/B only)")
    ap.add_argument("--freq-shift", type=float, default=0.0,
                    help="NCO mixer (apply_frequency_shift) fused into the FIR loads, Hz")
    ap.add_argument("--sample-rate", type=float, default=2e9, help="for --freq-shift (config 5: 2 GS/s)")
    ap.add_argument("--nchan", type=int, default=64)
    ap.add_argument("--branch-taps", type=int, default=16)
    ap.add_argument("--no-c2-leg", action="store_true",
                    help="skip the untimed-for-headline config-2 FIR+PSD leg after a c5 run")
    ap.add_argument("--c2-steps", type=int, default=10)
    ap.add_argument("--c2-samples", type=int, default=1 << 28)
    ap.add_argument("--launcher-selftest", default=None, help=argparse.SUPPRESS)
    ap.add_argument("--rehearse-one-gpu", action="store_true",
                    help="N ranks on cuda:0 over RCCL sockets (functional rehearsal of the N-GPU "
                         "path on a one-GPU box; not a scaling number)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        raise SystemExit(launch_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if args.launcher_selftest:
        return _launcher_selftest(args, world, rank, local)
    torch.cuda.set_device(local)
    dev = torch.device(f"cuda:{local}")
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    import vector_amd  # noqa: F401
    if args.workload == "pfb":
        return run_pfb(args, world, rank, local, dev)
    if args.workload == "sync":
        return run_sync(args, world, rank, local, dev)
    wdecim, wsamples, weak, wlabel = WORKLOADS[args.workload]
    decim = args.decim if args.decim is not None else wdecim
    if args.samples is not None:
        n = args.samples
    else:
        n = wsamples if weak else wsamples // world
    leg = run_chain_leg(args, n, decim, rank, world, local, dev, args.steps, args.warmup)
    elapsed, stages, stage_roof, check = leg["elapsed"], leg["stages"], leg["stage_roof"], leg["check"]
    roof, taps, tmpl = leg["roof"], leg["taps"], leg["tmpl"]
    N = world * n

    # north_star's own FIR+FFT target is quoted at config 2 (2**28 samples,
    # D = 1): after the headline's timed region, rank 0 runs that chain on its
    # GPU as a single-rank leg (not part of `value`) and reports its stages
    stages_c2 = None
    if rank == 0 and args.workload == "c5" and not args.no_c2_leg and args.decim is None:
        c2 = run_chain_leg(args, args.c2_samples, WORKLOADS["c2"][0], 0, 1, local, dev,
                           args.c2_steps, args.warmup)
        stages_c2 = dict(c2["stage_roof"], check=c2["check"], samples=args.c2_samples,
                         config=(f"BASELINE configs[1]: {args.c2_samples} samples, D = 1, "
                                 f"{args.ntaps} taps, {args.nfft}-pt PSD, {args.template}-sample "
                                 f"xcorr (single-rank leg after the timed region)"))
    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return
    ms_per_step = elapsed / args.steps * 1e3
    value = N / (elapsed / args.steps) / 1e6
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        cs = args.cpu_samples or (1 << 26)
        cpu = cpu_baseline(cs, taps, args.nfft, tmpl, decim)
        ncores, src = cpu_allowance()
        cpu["cores_available"] = ncores
        cpu["cores_source"] = src
        workers = args.cpu_workers or ncores
        # ~2 GB of numpy arrays per worker (a 2**25-sample chunk through
        # np.convolve / spectrogram / np.correlate complex128): stay within
        # half of the host memory available now
        try:
            import psutil
            cap = max(1, int(psutil.virtual_memory().available * 0.5 // (2 << 30)))
            if workers > cap:
                src += f"; {workers} -> {cap} workers for host memory"
                workers = cap
        except ImportError:
            pass
        if workers > 1:
            try:
                cpu["all_cores"] = cpu_baseline_allcores(cs // 2, taps, args.nfft, tmpl, workers,
                                                         decim)
                cpu["all_cores"]["cores_source"] = src
            except Exception as e:       # the GPU number stands without it
                cpu["all_cores"] = {"error": repr(e)[:200]}
    out = {
        "metric": METRIC, "value": round(value, 1), "unit": "Msamples/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True, "scaling": "weak" if (weak or args.samples is not None) else "strong",
        "vs_baseline": None, "dtype": "c64 (fp32)",
        "data": "synthetic IQ generated on device: 3 tones + CN(0,1) noise + QPSK preamble",
        "config": {"workload": (f"{wlabel}: {n} c64 samples/GPU, {args.ntaps}-tap overlap-save "
                                f"FIR, D={decim}, {args.nfft}-pt Hann PSD hop {args.nfft}, "
                                f"{args.template}-sample template xcorr (valid) + argmax"),
                   "name": args.workload, "samples_per_gpu": n, "total_samples": N,
                   "ntaps": args.ntaps, "decim": decim, "nfft": args.nfft,
                   "template": args.template,
                   "parallelism": f"time-chunk x{world} (RCCL halos)",
                   "freq_shift": args.freq_shift, "refine": not args.no_refine,
                   "refine_overlapped": not (args.no_refine or args.no_overlap_refine)},
        "roofline": roof,
        "cpu_baseline": cpu,
        "stages_ms": {k: round(v, 4) for k, v in stages.items()},
        "stages_ghz": leg["clocks"],
        "stages_roofline": stage_roof,
        "stages_roofline_c2": stages_c2,
        "check": check,
        "rccl_world": dist.get_world_size() if dist.is_initialized() else 1,
        "ranks": leg["ranks"],
    }
    if args.rehearse_one_gpu:
        out["rehearsal"] = (f"{world} ranks on one GPU over RCCL's socket transport: a functional "
                            f"run of the N-GPU path, not a scaling measurement")
    print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def run_sync(args, world, rank, local, dev):
    """BASELINE config 3: a 4096-sample QPSK preamble (SURVEY.md §8(d):
    default_rng(4096)) slid over a 2**30-sample synthetic stream planted at
    k0 = 123 456 789; valid correlation with the fused |c| argmax / sums
    (correlate_peak: cross_correlate_signals + find_correlation_peak,
    utils.py:1258-1342) on one GPU.  A step = one correlator launch + its
    partial finalize over the device-resident stream."""
    import ctypes as C
    from vector_amd import dsp
    if world != 1:
        raise SystemExit("--workload sync is BASELINE config 3 (one GPU)")
    n = args.samples if args.samples is not None else 1 << 30
    L = args.template
    _, pre, _ = design(args.ntaps, L)   # QPSK preamble, default_rng(4096)
    k0 = 123_456_789 if n > 123_456_789 + L else n // 3
    x = torch.empty(n, dtype=torch.complex64, device=dev)
    generate_chunk(x, 0, 20250718, pre, k0)
    xc = dsp.Correlator(pre, local)
    pk = torch.zeros(4, dtype=torch.float64, device=dev)
    torch.cuda.synchronize()
    for _ in range(args.warmup):
        xc(x, "valid", peak=pk)
    torch.cuda.synchronize()
    lib, h = xc.ctx.lib, xc.ctx.h
    lib.vsig_timing_reset(h)
    lib.vsig_timing_enable(h, 0 if args.no_kernel_timing else 1)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        xc(x, "valid", peak=pk)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    lib.vsig_timing_enable(h, 0)
    clocks = {} if args.no_kernel_timing else stage_clocks(lib, h, lambda: xc(x, "valid", peak=pk), 3)
    peak, idx, s1, s2 = dsp._read_peak(pk)
    nout = n - L + 1
    conf = dsp._confidence(peak, s1, s2, nout, 0.5)
    tot, cnt = C.c_double(), C.c_int64()
    lib.vsig_timing_read(h, b"xcorr", C.byref(tot), C.byref(cnt))
    roof = None
    stage = {}
    if cnt.value:
        ms = tot.value / cnt.value
        nbytes = 8 * n
        ach = nbytes / (ms * 1e-3) / 1e9
        M = xcorr_block(L)
        nb = -(-nout // (M - L + 1))
        flops = nb * (2 * 5 * M * np.log2(M) + 6 * M)
        tf = flops / (ms * 1e-3) / 1e12
        pmc = load_traffic(f"xcorr:n={n}:L={L}")
        roof = {"bound": "hbm", "kernel": "xcorr", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                "traffic": pmc["hbm_bytes_per_launch"] if pmc else None,
                "algorithmic_bytes": nbytes, "avg_launch_ms": round(ms, 4),
                "traffic_source": pmc["source"] if pmc else None}
        if pmc and "valu_issue_frac" in pmc:
            roof["valu_issue_frac"] = pmc["valu_issue_frac"]
        stage = {"xcorr": {"ms": round(ms, 4), "TFLOPs": round(tf, 2),
                           "valu_peak_TFLOPs": FP32_PEAK_TF, "valu_frac": round(tf / FP32_PEAK_TF, 4),
                           "M": M}}
        if "xcorr" in clocks:
            stage["xcorr"]["ghz"] = clocks["xcorr"]
    cpu = None
    if not args.no_cpu_baseline:
        from oracle import ref        # the CPU baseline leg only
        ns = args.cpu_samples or (1 << 24)
        xs = ref.synth_iq(ns, seed=99)
        t1 = time.perf_counter()
        c, lags = ref.cross_correlate_signals(pre, xs, "valid")
        ref.find_correlation_peak(c, lags)
        dt = time.perf_counter() - t1
        cpu = dict(value=round(ns / dt / 1e6, 3), unit="Msamples/s", cores=1, kind="port",
                   sample=(f"{ns} samples (2**{int(np.log2(ns))}) through np.correlate complex128 L={L} valid + "
                           f"find_correlation_peak, {dt:.2f} s, 1 thread (direct O(N L); the "
                           f"full 2**30 stream would take ~{n / (ns / dt) / 60:.0f} min)"),
                   seconds=round(dt, 3), cores_available=cpu_allowance()[0],
                   cores_source=cpu_allowance()[1])
    out = {
        "metric": "Msamples/s c64 through the sliding-correlation sync (BASELINE config 3)",
        "value": round(n / (elapsed / args.steps) / 1e6, 1), "unit": "Msamples/s",
        "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "c64 (fp32)",
        "data": "synthetic IQ generated on device: 3 tones + CN(0,1) noise + QPSK preamble",
        "config": {"workload": (f"BASELINE configs[2]: {L}-sample preamble over a {n}-sample "
                                f"c64 stream, valid correlation + argmax detect"),
                   "samples": n, "template": L, "parallelism": "1 GPU"},
        "roofline": roof, "cpu_baseline": cpu, "stages_roofline": stage,
        "check": {"lag": idx, "expected": k0, "ok": bool(idx == k0), "peak": round(peak, 3),
                  "confidence": round(conf, 4)},
    }
    print(json.dumps(out), flush=True)


def run_pfb(args, world, rank, local, dev):
    """BASELINE config 4: C-channel critically sampled PFB (prototype
    firwin(P*C, 1/C)) over a time-chunk-sharded capture; each rank gets the
    (P-1)*C-sample right halo from its neighbour over RCCL.  Default per-GPU
    chunk 2**29 samples (config 4's 2**31 over 4 GPUs)."""
    import ctypes as C
    import scipy.signal
    from vector_amd.shard import HipPfbBackend, PfbChain
    n = args.samples if args.samples is not None else 1 << 29
    nchan, P = args.nchan, args.branch_taps
    proto = scipy.signal.firwin(P * nchan, 1.0 / nchan).astype(np.float32)
    be = HipPfbBackend(proto, nchan, local)
    ch = PfbChain(n, proto, nchan, be, rank, world)
    generate_chunk(ch.x, rank * n, 20250718 + rank, np.zeros(0, np.complex64), -1)
    torch.cuda.synchronize()

    def barrier():
        if world > 1:
            dist.barrier()

    for _ in range(args.warmup):
        ch.step()
    torch.cuda.synchronize()
    barrier()
    lib, h = be.ctx.lib, be.ctx.h
    lib.vsig_timing_reset(h)
    lib.vsig_timing_enable(h, 0 if args.no_kernel_timing else 1)
    torch.cuda.synchronize()
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ch.step()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    barrier()
    lib.vsig_timing_enable(h, 0)
    clocks = {} if args.no_kernel_timing else stage_clocks(lib, h, ch.step, 3)
    barrier()
    elapsed = t1 - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    tot, cnt = C.c_double(), C.c_int64()
    lib.vsig_timing_read(h, b"pfb", C.byref(tot), C.byref(cnt))
    # spot check: the rank's frame 1 against the PFB's definition (pfb.hip header),
    # evaluated here in complex128 numpy
    xs = ch.x_ext[nchan: nchan + P * nchan].cpu().numpy().astype(np.complex128)
    z = (proto.astype(np.float64) * xs).reshape(P, nchan).sum(axis=0)
    want = np.fft.fft(z)
    got = ch.frames()[1].cpu().numpy()
    err = float(np.abs(got - want).max() / np.abs(want).max())
    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return
    N = world * n
    roof = None
    if cnt.value:
        ms = tot.value / cnt.value
        nbytes = 8 * (n + ch.rhalo) + 8 * ch.nframes * nchan
        ach = nbytes / (ms * 1e-3) / 1e9
        pmc = load_traffic(f"pfb:n={n}:nchan={nchan}:P={P}")
        roof = {"bound": "hbm", "kernel": "pfb", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                "traffic": pmc["hbm_bytes_per_launch"] if pmc else None,
                "algorithmic_bytes": nbytes, "avg_launch_ms": round(ms, 4),
                "traffic_source": pmc["source"] if pmc else None}
        if "pfb" in clocks:
            roof["ghz"] = clocks["pfb"]
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        from oracle import ref        # the CPU baseline leg only
        ns = args.cpu_samples or (1 << 27)
        xs = ref.synth_iq(ns, seed=99)
        t0 = time.perf_counter()
        ref.pfb_channelize(xs, proto, nchan)
        dt = time.perf_counter() - t0
        cpu = dict(value=round(ns / dt / 1e6, 3), unit="Msamples/s", cores=1, kind="port",
                   sample=f"{ns} samples through oracle pfb_channelize (numpy, complex128), "
                          f"{dt:.2f} s", seconds=round(dt, 3))
    out = {
        "metric": f"Msamples/s c64 through {nchan}-channel PFB channelizer (BASELINE config 4)",
        "value": round(N / (elapsed / args.steps) / 1e6, 1), "unit": "Msamples/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "c64 (fp32)",
        "data": "synthetic IQ generated on device: 3 tones + CN(0,1) noise",
        "config": {"workload": (f"BASELINE configs[3]: {n} c64 samples/GPU, {nchan}-channel "
                                f"critically sampled PFB, {P * nchan}-tap firwin prototype"),
                   "samples_per_gpu": n, "total_samples": N, "nchan": nchan, "branch_taps": P,
                   "parallelism": f"time-chunk x{world} (RCCL right halo {P * nchan - nchan})"},
        "roofline": roof, "cpu_baseline": cpu,
        "check": {"frame1_rel_err": err, "ok": err < 1e-5},
        "rccl_world": dist.get_world_size() if dist.is_initialized() else 1,
    }
    if args.rehearse_one_gpu:
        out["rehearsal"] = (f"{world} ranks on one GPU over RCCL's socket transport: a functional "
                            f"run of the N-GPU path, not a scaling measurement")
    print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
