"""Benchmark: Msamples/s of complex64 IQ through the FIR -> (decimate) -> FFT-PSD
-> xcorr-sync chain on 1..N MI355X GPUs, with the dominant kernel's achieved
HBM bandwidth against the roofline and the CPU reference path beside it.

Workload (BASELINE.json configs[1], extended with the sync stage the metric
names): every rank owns a contiguous 2**28-sample (256 Msample, 2 GiB) time
chunk of one long synthetic capture; 255-tap overlap-save FIR, D = 1;
8192-point Hann PSD, hop 8192; 4096-sample template valid correlation with a
fused |c| argmax.  Weak scaling: N GPUs process an N x 256 Msample capture
(N = 8 is BASELINE config 5's 2**31 samples), exchanging only the FIR /
correlation halos and 32-byte peak records over RCCL.

  python bench.py [--gpus N --steps K --warmup W]
  python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...
  python bench.py --workload pfb      # BASELINE config 4 (64-channel PFB), not the headline
  python bench.py --workload sync     # BASELINE config 3 (4096-sample preamble over 2**30)
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


def cpu_baseline(samples, taps, nfft, tmpl):
    """The reference's CPU path (oracle: np.convolve / scipy.signal.spectrogram /
    np.correlate, single-threaded numpy) timed on a bounded sample."""
    from oracle import ref
    x = ref.synth_iq(samples, seed=99)
    t0 = time.perf_counter()
    y = ref.fir_filter(x, taps, 1)
    ref.spectrum(y, 1.0, "hann", nfft, 0, nfft)
    c, lags = ref.cross_correlate_signals(tmpl, y, "valid")
    ref.find_correlation_peak(c, lags)
    dt = time.perf_counter() - t0
    return dict(value=round(samples / dt / 1e6, 3), unit="Msamples/s", cores=1, kind="port",
                sample=(f"{samples} samples (2**{int(np.log2(samples))}) of the same chain: "
                        f"np.convolve {len(taps)} taps, scipy spectrogram nfft={nfft}, "
                        f"np.correlate complex128 L={len(tmpl)} valid + find_correlation_peak; "
                        f"{dt:.2f} s, 1 thread"),
                seconds=round(dt, 3))


def cpu_baseline_allcores(samples, taps, nfft, tmpl, workers):
    """The same CPU chain as cpu_baseline on `workers` processes, one time
    chunk each with its halos (SURVEY.md §8(d)'s all-cores variant); value =
    all chunks' samples / the wall time of the parallel map (worker start-up
    and imports excluded by a warm-up map)."""
    import multiprocessing as mp
    from oracle import ref
    ctx = mp.get_context("spawn")       # fresh interpreters: no GPU state in the workers
    jobs = [(samples, 1000 + w, taps, nfft, tmpl) for w in range(workers)]
    with ctx.Pool(workers) as pool:
        pool.map(ref.chain_chunk_seconds, [(1 << 12, w, taps, nfft, tmpl) for w in range(workers)])
        t0 = time.perf_counter()
        secs = pool.map(ref.chain_chunk_seconds, jobs)
        dt = time.perf_counter() - t0
    return dict(value=round(workers * samples / dt / 1e6, 3), unit="Msamples/s", cores=workers,
                kind="port",
                sample=(f"{workers} processes x {samples} samples (2**{int(np.log2(samples))}) of "
                        f"the chain with halos, {dt:.2f} s wall (per-chunk {min(secs):.2f}-"
                        f"{max(secs):.2f} s)"),
                seconds=round(dt, 3))


def xcorr_block(L, forced):
    """Overlap-save block size the correlator plans for a template of L
    (vsig_api.hip os_size_xcorr, unless forced with --xcorr-m)."""
    if forced:
        return forced
    return 4096 if L <= 1024 else 8192 if L <= 2048 else 16384


def load_traffic(key):
    """Measured HBM bytes per launch from a committed rocprofv3 --pmc summary
    (profiles/pmc_*.json, corrected as MI355X_MICROARCH.md §HBM prescribes)."""
    import glob
    best = None
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_*.json"))):
        try:
            d = json.load(open(p))
        except Exception:
            continue
        if d.get("config_key") == key:
            best = d
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--samples", type=int, default=1 << 28, help="input samples per GPU")
    ap.add_argument("--ntaps", type=int, default=255)
    ap.add_argument("--decim", type=int, default=1)
    ap.add_argument("--nfft", type=int, default=8192)
    ap.add_argument("--template", type=int, default=4096)
    ap.add_argument("--cpu-samples", type=int, default=1 << 22)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-workers", type=int, default=16,
                    help="processes for the all-cores CPU baseline (the GPU box's CPU share is 16)")
    ap.add_argument("--no-kernel-timing", action="store_true")
    ap.add_argument("--pipeline", type=int, default=1,
                    help="sub-chunks per step: FIR / PSD / xcorr overlap on three HIP streams")
    ap.add_argument("--serial", action="store_true",
                    help="run the --pipeline sub-chunks in order on one stream (cache reuse)")
    for k in ("psd_variant", "fir_variant", "xcorr_variant", "fir_m", "xcorr_m", "fir_psd_variant", "psd_grid"):
        ap.add_argument("--" + k.replace("_", "-"), type=int, default=None)
    ap.add_argument("--freq-shift", type=float, default=0.0,
                    help="NCO mixer (apply_frequency_shift) fused into the FIR loads, Hz")
    ap.add_argument("--sample-rate", type=float, default=2e9, help="for --freq-shift (config 5: 2 GS/s)")
    ap.add_argument("--three-streams", action="store_true",
                    help="FIR / PSD / xcorr on their own HIP streams (default: one stream)")
    ap.add_argument("--fuse", action="store_true",
                    help="FIR and PSD in one fused launch (D=1, nfft 8192; default: two launches)")
    ap.add_argument("--workload", choices=("chain", "pfb", "sync"), default="chain",
                    help="chain: the headline FIR->PSD->xcorr metric; pfb: config 4 channelizer; "
                         "sync: config 3 preamble correlation over 2**30 samples")
    ap.add_argument("--nchan", type=int, default=64)
    ap.add_argument("--branch-taps", type=int, default=16)
    ap.add_argument("--pfb-variant", type=int, default=None)
    ap.add_argument("--pfb-fpg", type=int, default=None)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: launch N>1 with "
                         "python -m torch.distributed.run --nproc-per-node N bench.py --gpus N")
    torch.cuda.set_device(local)
    dev = torch.device(f"cuda:{local}")
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    import vector_amd  # noqa: F401
    if args.workload == "pfb":
        return run_pfb(args, world, rank, local, dev)
    if args.workload == "sync":
        return run_sync(args, world, rank, local, dev)
    from vector_amd.shard import ChainConfig, HipBackend, StreamChain

    n = args.samples
    taps, pre, tmpl = design(args.ntaps, args.template, args.decim)
    from vector_amd._lib import get_context
    ctx0 = get_context(local)
    for k in ("psd_variant", "fir_variant", "xcorr_variant", "fir_m", "xcorr_m", "fir_psd_variant", "psd_grid"):
        v = getattr(args, k)
        if v is not None:
            ctx0.check(ctx0.lib.vsig_set_option(ctx0.h, k.encode(), v), k)
    cfg = ChainConfig(n_local=n, taps=taps, decim=args.decim, nfft=args.nfft, template=tmpl,
                      pipeline=args.pipeline, serial=args.serial, fuse=args.fuse,
                      one_stream=not args.three_streams,
                      freq_shift=args.freq_shift, sample_rate=args.sample_rate)
    be = HipBackend(cfg, local)
    chain = StreamChain(cfg, be, rank, world)
    N = world * n
    ny_total = N // args.decim
    k0 = (ny_total // 2 + 12_345) * args.decim     # global input sample of the preamble
    if args.freq_shift:   # plant the preamble so that it leaves the mixer unrotated
        ph = 2 * np.pi * args.freq_shift * ((k0 + np.arange(len(pre))) / args.sample_rate)
        pre = (pre * np.exp(-1j * ph)).astype(np.complex64)
    generate_chunk(chain.x, rank * n, 20250718 + rank, pre, k0)
    torch.cuda.synchronize()

    def barrier():
        if world > 1:
            dist.barrier()

    for _ in range(args.warmup):
        chain.step()
    torch.cuda.synchronize()
    barrier()
    lib, h = be.ctx.lib, be.ctx.h
    lib.vsig_timing_reset(h)
    lib.vsig_timing_enable(h, 0 if args.no_kernel_timing else 1)
    torch.cuda.synchronize()
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        chain.step()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    barrier()
    lib.vsig_timing_enable(h, 0)
    elapsed = t1 - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # per-kernel durations from HIP events on the launch stream
    import ctypes as C
    stages = {}
    for name in ("fir", "psd", "fir_psd", "xcorr"):
        tot, cnt = C.c_double(), C.c_int64()
        lib.vsig_timing_read(h, name.encode(), C.byref(tot), C.byref(cnt))
        if cnt.value:
            stages[name] = tot.value / cnt.value
    ny = n // args.decim
    # fir_psd (fused): x read + y written + Sxx written; the PSD's re-read of y
    # is served by L2 / the Infinity Cache (PMC traffic in profiles/ checks it)
    bytes_per_launch = {"fir": 8 * n + 8 * ny, "psd": 8 * ny + 4 * ny,
                        "fir_psd": 8 * n + 8 * ny + 4 * ny, "xcorr": 8 * (ny + chain.yhalo)}
    m, lag, s1, s2, nout = chain.global_peak()
    check = {"sync_lag": lag, "expected": k0 // args.decim, "ok": bool(lag == k0 // args.decim)}

    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return
    ms_per_step = elapsed / args.steps * 1e3
    value = N / (elapsed / args.steps) / 1e6
    roof = None
    if stages:
        dom = max(stages, key=lambda k: stages[k])
        achieved = bytes_per_launch[dom] / (stages[dom] * 1e-3) / 1e9
        key = f"{dom}:n={n}:ntaps={args.ntaps}:decim={args.decim}:nfft={args.nfft}:L={args.template}"
        pmc = load_traffic(key)
        roof = {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": pmc["hbm_bytes_per_launch"] if pmc else None,
                "algorithmic_bytes": bytes_per_launch[dom],
                "avg_launch_ms": round(stages[dom], 4),
                "traffic_source": pmc["source"] if pmc else None}
        if pmc and "valu_issue_frac" in pmc:
            # the correlator is VALU-bound: its issue utilisation from the same PMC pass
            roof["valu_issue_frac"] = pmc["valu_issue_frac"]
    # every stage against its own roof: HBM bytes for all three, and for the
    # correlator (not HBM-bound) the FP32 vector roof with the standard
    # 5 N log2 N FFT flop count (2 FFTs + the spectrum multiply per block)
    stage_roof = {}
    for k, ms in stages.items():
        gbs = bytes_per_launch[k] / (ms * 1e-3) / 1e9
        stage_roof[k] = {"ms": round(ms, 4), "bytes": bytes_per_launch[k], "GBs": round(gbs, 1),
                         "hbm_frac": round(gbs / HBM_PEAK_GBS, 4)}
        pk = load_traffic(f"{k}:n={n}:ntaps={args.ntaps}:decim={args.decim}:nfft={args.nfft}:"
                          f"L={args.template}")
        if pk and "valu_issue_frac" in pk:
            stage_roof[k]["valu_issue_frac"] = pk["valu_issue_frac"]
    if "xcorr" in stages:
        M = xcorr_block(args.template, args.xcorr_m)
        L = args.template
        hop = M - L + 1
        nb = -(-(ny + chain.yhalo - L + 1) // hop)
        flops = nb * (2 * 5 * M * np.log2(M) + 6 * M)
        tf = flops / (stages["xcorr"] * 1e-3) / 1e12
        stage_roof["xcorr"].update({"flops": int(flops), "TFLOPs": round(tf, 2),
                                    "valu_peak_TFLOPs": FP32_PEAK_TF,
                                    "valu_frac": round(tf / FP32_PEAK_TF, 4), "M": M})
    # north_star's FIR+FFT target on SURVEY.md §8(d) C2's unfused byte count
    # (28 B/sample: filter() writes y, spectrum() reads it); with the fused
    # kernel the HBM bytes actually moved are 20 B/sample (stage "fir_psd")
    fp_ms = (stages["fir"] + stages["psd"]) if ("fir" in stages and "psd" in stages) \
        else stages.get("fir_psd")
    if fp_ms:
        b = bytes_per_launch["fir"] + bytes_per_launch["psd"]
        t = fp_ms * 1e-3
        stage_roof["fir+psd"] = {"ms": round(fp_ms, 4), "GBs": round(b / t / 1e9, 1),
                                 "hbm_frac": round(b / t / 1e9 / HBM_PEAK_GBS, 4),
                                 "bytes_basis": "28 B/sample (unfused FIR 16 + PSD 12)",
                                 "fused": "fir_psd" in stages}
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.cpu_samples, taps, args.nfft, tmpl)
        cpu["cores_available"] = len(os.sched_getaffinity(0))
        if args.cpu_workers > 1:
            try:
                cpu["all_cores"] = cpu_baseline_allcores(args.cpu_samples // 2, taps, args.nfft,
                                                         tmpl, args.cpu_workers)
            except Exception as e:       # the GPU number stands without it
                cpu["all_cores"] = {"error": repr(e)[:200]}
    out = {
        "metric": METRIC, "value": round(value, 1), "unit": "Msamples/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "c64 (fp32)",
        "data": "synthetic IQ generated on device: 3 tones + CN(0,1) noise + QPSK preamble",
        "config": {"workload": (f"BASELINE configs[1] chain + sync: {n} c64 samples/GPU, "
                                f"{args.ntaps}-tap overlap-save FIR, D={args.decim}, "
                                f"{args.nfft}-pt Hann PSD hop {args.nfft}, "
                                f"{args.template}-sample template xcorr (valid) + argmax"),
                   "samples_per_gpu": n, "total_samples": N, "ntaps": args.ntaps,
                   "decim": args.decim, "nfft": args.nfft, "template": args.template,
                   "parallelism": f"time-chunk x{world} (RCCL halos)",
                   "pipeline": args.pipeline, "serial": args.serial, "fused": chain.fused,
                   "freq_shift": args.freq_shift},
        "roofline": roof,
        "cpu_baseline": cpu,
        "stages_ms": {k: round(v, 4) for k, v in stages.items()},
        "stages_roofline": stage_roof,
        "check": check,
    }
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
    n = args.samples if args.samples != 1 << 28 else 1 << 30
    L = args.template
    from oracle import ref            # preamble generator (same seed as the oracle's goldens)
    pre = ref.qpsk_preamble(L, seed=4096)
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
        M = xcorr_block(L, args.xcorr_m)
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
    cpu = None
    if not args.no_cpu_baseline:
        ns = 1 << 21
        xs = ref.synth_iq(ns, seed=99)
        t1 = time.perf_counter()
        c, lags = ref.cross_correlate_signals(pre, xs, "valid")
        ref.find_correlation_peak(c, lags)
        dt = time.perf_counter() - t1
        cpu = dict(value=round(ns / dt / 1e6, 3), unit="Msamples/s", cores=1, kind="port",
                   sample=(f"{ns} samples (2**21) through np.correlate complex128 L={L} valid + "
                           f"find_correlation_peak, {dt:.2f} s, 1 thread (direct O(N L); the "
                           f"full 2**30 stream would take ~{n / (ns / dt) / 60:.0f} min)"),
                   seconds=round(dt, 3), cores_available=len(os.sched_getaffinity(0)))
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
    n = args.samples if args.samples != 1 << 28 else 1 << 29
    nchan, P = args.nchan, args.branch_taps
    proto = scipy.signal.firwin(P * nchan, 1.0 / nchan).astype(np.float32)
    be = HipPfbBackend(proto, nchan, local)
    for k in ("pfb_variant", "pfb_fpg"):
        v = getattr(args, k)
        if v is not None:
            be.ctx.check(be.ctx.lib.vsig_set_option(be.ctx.h, k.encode(), v), k)
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
    elapsed = t1 - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    tot, cnt = C.c_double(), C.c_int64()
    lib.vsig_timing_read(h, b"pfb", C.byref(tot), C.byref(cnt))
    # spot check: the rank's frame 1 against the definition (oracle is test infra)
    from oracle import ref
    xs = ch.x_ext[: nchan + P * nchan].cpu().numpy()
    want = ref.pfb_channelize(xs, proto, nchan)[:, 1]
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
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        ns = 1 << 22
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
    }
    print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
