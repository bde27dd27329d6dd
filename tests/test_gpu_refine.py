"""Exact argmax of the correlators (refine.hip) against numpy's complex128
argmax, find_correlation_peak (utils.py:1321-1325) over cross_correlate_signals
(utils.py:1279-1285).

The fp32 FFT correlation is ~1e-8 * |p| |s_segment| from the exact sums, so
near-ties closer than that were decided by rounding noise before this pass.
The reference's own tone data (tests/golden/tone_transplant.npz, made by
tests/golden/make_golden.py from data/packet_*.mat and
data/fixed_test_vector.mat) have top-2 |c|^2 gaps of 1e-13 .. 7e-12
(relative), and a tone against itself ties in exact arithmetic (40 005 of
48 195 outputs within 1e-12 of the max): numpy's answer there is decided by the
rounding of its own evaluation order.  The refine evaluates every output that
can be the maximum in that order (OpenBLAS zdotu's accumulator layout and
numpy's complex abs, oracle/npdot.c, pinned against numpy in
tests/test_npdot_cpu.py), so lag, location and peak value equal the
reference's bit for bit.
"""
import numpy as np
import pytest
import torch

from conftest import golden
from oracle import ref

pytestmark = pytest.mark.gpu


def _status(gpu):
    return gpu.dsp.refine_status()


@pytest.mark.parametrize("i", [1, 2, 3, 4, 5, 6])
def test_tone_packet_in_vector_exact_lag(gpu, i):
    g = golden("tone_transplant.npz")
    vec, seg = g["vector"], g[f"seg{i}"]
    want_lag, want_val, want_conf = g[f"vec{i}_peak"]
    # stored array (complex128, refined outputs patched in) + find_correlation_peak
    c, lags = gpu.cross_correlate_signals(seg, vec)
    assert c.dtype == np.complex128
    lag, val, conf = gpu.find_correlation_peak(c, lags)
    assert lag == want_lag
    assert int(np.argmax(np.abs(c))) == int(g[f"vec{i}_argmax"])
    assert val == want_val                       # numpy's |c| to the bit
    assert conf == pytest.approx(want_conf, rel=1e-5, abs=1e-7)
    # fused (no array)
    lag2, val2, conf2 = gpu.correlate_peak(seg, vec)
    assert lag2 == want_lag
    assert val2 == want_val
    assert _status(gpu)[0] == 0


@pytest.mark.parametrize("i", [1, 3])
def test_tone_packet_self_ties(gpu, i):
    """A tone against itself: ~40 000 exact ties; numpy's pick (index 14 523 /
    36 418 of 48 195) is reproduced, fused and through the stored array."""
    g = golden("tone_transplant.npz")
    pk, seg = g[f"packet{i}"], g[f"seg{i}"]
    want_lag, want_val, want_conf = g[f"pkt{i}_peak"]
    lag, val, conf = gpu.correlate_peak(seg, pk)
    st, cand = _status(gpu)
    print(f"packet {i}: lag {int(lag)} (numpy {int(want_lag)}), {cand} candidate items, "
          f"{int(g[f'pkt{i}_nearmax'])} outputs within 1e-12 of the max")
    assert st == 0
    assert lag == want_lag
    assert val == want_val
    assert conf == pytest.approx(want_conf, rel=1e-5, abs=1e-7)
    c, lags = gpu.cross_correlate_signals(seg, pk)
    assert int(np.argmax(np.abs(c))) == int(g[f"pkt{i}_argmax"])
    assert gpu.find_correlation_peak(c, lags)[0] == want_lag


@pytest.mark.parametrize("i", [1, 3])
def test_tone_find_packet_location(gpu, i):
    """find_packet_location_in_vector on the reference's data (utils.py:1372-1434):
    the vector lag and the packet self-tie both equal numpy's, so the location
    is the reference's."""
    g = golden("tone_transplant.npz")
    vec, pk, seg = g["vector"], g[f"packet{i}"], g[f"seg{i}"]
    loc, ploc, conf = gpu.find_packet_location_in_vector(vec, pk, seg)
    want = g[f"loc{i}"]
    assert loc == want[0]
    assert ploc == want[1] == 0
    assert conf == pytest.approx(want[2], rel=1e-5, abs=1e-7)


@pytest.mark.parametrize("L,ns,mode,swapped,dt", [
    (4096, 60_000, "valid", False, np.complex64), (4096, 60_000, "full", False, np.complex128),
    (777, 20_000, "full", False, np.complex128), (1500, 30_000, "full", True, np.complex128),
    (3000, 3000, "same", False, np.complex128),
    (12_000, 50_000, "valid", False, np.complex128),   # > 10000 terms: OpenBLAS thread split
    (20_000, 45_000, "full", True, np.complex64), (5, 3000, "full", False, np.complex128)])
def test_numpy_order_value_bit_exact(gpu, L, ns, mode, swapped, dt):
    """Planted template in noise: the refined peak (fused record and the patched
    complex128 array) is numpy's complex128 value and |c| to the bit."""
    rng = np.random.default_rng(L + ns)
    t = (rng.standard_normal(L) + 1j * rng.standard_normal(L)).astype(dt)
    s = (rng.standard_normal(ns) + 1j * rng.standard_normal(ns)).astype(dt)
    k0 = min(ns // 3, ns - L)
    s[k0:k0 + L] += t
    a, b = (s, t) if swapped else (t, s)
    r, rl = ref.cross_correlate_signals(a, b, mode)
    want = ref.find_correlation_peak(r, rl)
    lag, val, _ = gpu.correlate_peak(a, b, mode)
    assert lag == want[0]
    assert val == want[1]
    c, lags = gpu.cross_correlate_signals(a, b, mode)
    k = int(np.argmax(np.abs(c)))
    assert lags[k] == want[0]
    assert c[k] == r[k] and np.abs(c)[k] == want[1]


def test_exact_ties_lowest_index(gpu):
    """A periodic stream and one period as template: the correlation peaks at
    every period with bit-identical exact sums; np.argmax takes the first."""
    P, reps = 1500, 40
    per = ref.qpsk_preamble(P, seed=5)
    s = np.tile(per, reps)
    for mode in ("valid", "full"):
        lag, _, _ = gpu.correlate_peak(per, s, mode)
        want = ref.find_correlation_peak(*ref.cross_correlate_signals(per, s, mode))
        assert lag == want[0]
        c, lags = gpu.cross_correlate_signals(per, s, mode)
        assert gpu.find_correlation_peak(c, lags)[0] == want[0]


@pytest.mark.parametrize("ratio", [1 + 1e-9, 1 - 1e-9])
def test_near_tie_below_fp32_resolution(gpu, ratio):
    """Two copies of the preamble with amplitudes 1 and `ratio` (1e-9 apart,
    100x below the fp32 correlation's resolution): the larger one wins."""
    L, n = 2048, 200_000
    pre = ref.qpsk_preamble(L, seed=9)
    s = np.zeros(n, np.complex128)                    # noise-free around the copies
    s[:20_000] = 0.01 * ref.synth_iq(20_000, seed=10)
    s[50_000:50_000 + L] += pre
    s[150_000:150_000 + L] += ratio * pre.astype(np.complex128)   # (complex64 * float stays complex64)
    want = ref.find_correlation_peak(*ref.cross_correlate_signals(pre, s, "valid"))
    lag, val, _ = gpu.correlate_peak(pre, s, "valid")
    assert lag == want[0] == (150_000 if ratio > 1 else 50_000)
    assert val == want[1]


def test_streaming_correlator_refined(gpu):
    """The chain's streaming Correlator (device stream, fused peak record) is
    refined too: exact lag on two nearly equal planted copies."""
    L, n = 4096, 1 << 20
    pre = ref.qpsk_preamble(L, seed=11)
    s = ref.synth_iq(n, seed=12)
    s[100_000:100_000 + L] += 3 * pre
    s[700_000:700_000 + L] += np.complex64(3 * (1 + 3e-7)) * pre
    want = ref.xcorr_peak(s, pre, "valid")
    xc = gpu.Correlator(pre)
    _, pk = xc(torch.from_numpy(s).cuda(), "valid")
    peak, idx, s1, s2 = gpu.dsp._read_peak(pk)
    assert idx == want[1]
    assert peak == want[2]


def test_refine_cap_opt_in_and_off(gpu):
    """Default: no cap (every candidate evaluated, status 0).  An explicit
    'refine_cap' below the candidate count leaves the record fp32 (status 1, the
    numpy front end warns); refine off: no pass at all."""
    import ctypes as C
    ctx = gpu.get_context()
    tone = np.exp(2j * np.pi * 0.01 * np.arange(300_000)).astype(np.complex64)
    gpu.correlate_peak(tone[:1000], tone, "valid")
    assert _status(gpu)[0] == 0
    ctx.check(ctx.lib.vsig_set_option(ctx.h, b"refine_cap", 8192), "cap")
    try:
        with pytest.warns(RuntimeWarning, match="refine_cap"):
            gpu.correlate_peak(tone[:1000], tone, "valid")
        assert _status(gpu)[0] == 1
    finally:
        ctx.check(ctx.lib.vsig_set_option(ctx.h, b"refine_cap", 0), "cap")
    ctx.check(ctx.lib.vsig_set_option(ctx.h, b"refine", 0), "off")
    try:
        gpu.correlate_peak(tone[:1000], tone[:5000], "valid")
        assert _status(gpu)[0] == 2
    finally:
        ctx.check(ctx.lib.vsig_set_option(ctx.h, b"refine", 1), "on")
    v = C.c_int()
    ctx.check(ctx.lib.vsig_get_option(ctx.h, b"refine", C.byref(v)), "get")
    assert v.value == 1
    ctx.check(ctx.lib.vsig_get_option(ctx.h, b"refine_cap", C.byref(v)), "get")
    assert v.value == 0


def _flat_tone(g):
    dur, sr, f = g["a_args"]
    tone = ref.generate_sample_packet(float(dur), float(sr), float(f))
    import hashlib
    assert hashlib.sha256(tone.tobytes()).hexdigest() == str(g["a_sha"]), \
        "numpy regenerated a different tone than the golden's"
    return tone


def test_flat_tone_2e21_exact(gpu):
    """The reference's flat case at scale (refine_flat.npz (a), made by the
    reference's cross_correlate_signals + find_correlation_peak): a 2^21-sample
    tone against its first 4096 samples, 'full' -- 2 093 057 outputs within
    1e-12 of the max, every full-overlap output in the refine band.  numpy's
    argmax (decided by the rounding of its own sums) and |c| exactly, fused and
    through the stored complex128 array."""
    g = golden("refine_flat.npz")
    tone = _flat_tone(g)
    seg = tone[:4096]
    want_lag, want_val, want_conf = g["a_peak"]
    lag, val, conf = gpu.correlate_peak(seg, tone)
    st, cand = _status(gpu)
    print(f"2^21 tone: {cand} candidate items, lag {int(lag)} (numpy {int(want_lag)})")
    assert st == 0
    assert lag == want_lag
    assert val == want_val
    assert conf == pytest.approx(want_conf, rel=1e-5, abs=1e-7)
    c, lags = gpu.cross_correlate_signals(seg, tone)
    assert int(np.argmax(np.abs(c))) == int(g["a_argmax"])
    lag2, val2, conf2 = gpu.find_correlation_peak(c, lags)
    assert (lag2, val2) == (want_lag, want_val)
    assert conf2 == pytest.approx(want_conf, rel=1e-5, abs=1e-7)


def test_periodic_tone_packet_vector_exact(gpu):
    """refine_flat.npz (b): 30 instances of the reference's data/packet_1.mat in a
    vector built as the reference's GUI builds it (unified_gui.py:1712,
    1755-1769), searched with the packet's first 4096 samples: numpy's lag, |c|
    and find_packet_location_in_vector result exactly."""
    g = golden("refine_flat.npz")
    t = golden("tone_transplant.npz")
    period, reps, total = (int(v) for v in g["b_args"])
    pk, seg = t["packet1"], t["seg1"]
    vec = ref.periodic_vector(pk.astype(np.complex64), period, total)
    import hashlib
    assert hashlib.sha256(vec.tobytes()).hexdigest() == str(g["b_sha"])
    want_lag, want_val, want_conf = g["b_peak"]
    lag, val, conf = gpu.correlate_peak(seg, vec)
    assert _status(gpu)[0] == 0
    assert lag == want_lag
    assert val == want_val
    assert conf == pytest.approx(want_conf, rel=1e-5, abs=1e-7)
    c, lags = gpu.cross_correlate_signals(seg, vec)
    assert int(np.argmax(np.abs(c))) == int(g["b_argmax"])
    loc = gpu.find_packet_location_in_vector(vec, pk, seg)
    want = g["b_loc"]
    assert loc[0] == want[0] and loc[1] == want[1]
    assert loc[2] == pytest.approx(want[2], rel=1e-5, abs=1e-7)


def test_flat_valid_confidence_exact(gpu):
    """refine_flat.npz (c): a 1000-sample tone template over a 20000-sample tone,
    'valid' -- |c| is flat, numpy's std_corr (1.07e-13) is rounding noise and
    its confidence 0.318 follows from it.  Fused: the fp32 sums cannot resolve
    that std, so every output is re-evaluated in numpy's order and numpy's
    two-pass statistics are formed from them (vsig_correlate_stats_dev); from
    the stored array: vsig_abs_stats_dev.  Both equal numpy's to the bit."""
    g = golden("refine_flat.npz")
    tone = g["c_tone"]
    tm = tone[:1000]
    want_lag, want_val, want_conf = g["c_peak"]
    lag, val, conf = gpu.correlate_peak(tm, tone, "valid")
    assert (lag, val) == (want_lag, want_val)
    assert conf == want_conf
    c, lags = gpu.cross_correlate_signals(tm, tone, "valid")
    assert np.array_equal(np.abs(c), g["c_abs"])         # every output numpy's (dense refine)
    assert gpu.find_correlation_peak(c, lags) == (want_lag, want_val, want_conf)


@pytest.mark.parametrize("na,nv,mode,dt", [
    (20_000, 1000, "full", np.complex128),     # a slides (the template is the shorter operand)
    (1000, 20_000, "full", np.complex128),     # v slides (np.correlate's swapped order)
    (1000, 20_000, "valid", np.complex64),
    (30_000, 3000, "same", np.complex64),
    (40_000, 12_000, "valid", np.complex128),  # > 10000 terms: OpenBLAS's thread split
    (12_000, 40_000, "full", np.complex64)])
def test_flat_dense_every_geometry(gpu, na, nv, mode, dt):
    """The dense numpy-order form on a flat |c| (every full-overlap output in
    the band) in both operand orders, every mode, both precisions and sums
    over 10000 terms: the argmax, |c| and complex128 value equal numpy's bit
    for bit (np.correlate complex128 = the reference's arithmetic), the
    confidence to 1e-5 (north_star's float bar)."""
    t = np.arange(max(na, nv))
    tone = np.exp(2j * np.pi * 0.0123 * t).astype(dt)
    a, v = tone[:na], tone[:nv]
    # cross_correlate_signals(signal1=v, signal2=a) = np.correlate(a, v) in complex128
    r = np.correlate(a.astype(np.complex128), v.astype(np.complex128), mode)
    ar = np.abs(r)
    c, lags = gpu.cross_correlate_signals(v, a, mode)
    assert _status(gpu)[0] == 0
    k = int(np.argmax(np.abs(c)))
    assert k == int(np.argmax(ar))
    assert np.abs(c)[k] == ar.max() and c[k] == r[k]
    try:
        want = ref.find_correlation_peak(r, lags)
    except IndexError:                 # the reference's lag-axis quirks ('same' / long signal1)
        with pytest.raises(IndexError):
            gpu.correlate_peak(v, a, mode)
        return
    got = gpu.correlate_peak(v, a, mode)
    assert got[0] == want[0]
    assert got[1] == want[1]
    # the confidence from the fused fp32 sums (the ramps of 'full' / 'same' give
    # a wide spread) or, for a flat |c|, numpy's own statistics
    assert got[2] == pytest.approx(want[2], rel=1e-5, abs=1e-7)
    lag2, val2, conf2 = gpu.find_correlation_peak(c, lags)
    assert (lag2, val2) == want[:2]
    assert conf2 == pytest.approx(want[2], rel=1e-5, abs=1e-7)


@pytest.mark.parametrize("n", [1, 7, 100, 8192, 8193, 50_000, (1 << 20) + 3])
def test_abs_stats_numpy_order(gpu, n):
    """vsig_abs_stats_dev = np.mean(np.abs(a)), np.std(np.abs(a)) bit for bit
    (complex128 and float64)."""
    import torch
    rng = np.random.default_rng(n)
    a = (rng.standard_normal(n) + 1j * rng.standard_normal(n)) * 10 ** rng.uniform(-3, 3, n)
    ctx = gpu.get_context()
    for arr, code in ((a, "c128"), (a.real.copy(), "f64")):
        t = torch.from_numpy(arr).cuda()
        m, sd = gpu.dsp._abs_stats(t, code, ctx)
        assert m == np.mean(np.abs(arr))
        assert sd == np.std(np.abs(arr))


@pytest.mark.parametrize("L,ns,mode", [(10_000, 60_000, "valid"), (20_000, 90_000, "full"),
                                       (12_000, 7_000, "full")])
def test_long_template_correlator(gpu, L, ns, mode):
    """Streaming Correlator with templates longer than 8192 (one pass per
    8192-sample chunk): c (out=) and the refined peak record against np.correlate,
    including a stream shorter than the template (full mode)."""
    pre = ref.qpsk_preamble(L, seed=L)
    s = ref.synth_iq(ns, seed=ns)
    k0 = ns // 3
    if ns >= L:
        s[k0:k0 + L] += pre
    xc = gpu.Correlator(pre)
    nout = ns - L + 1 if mode == "valid" else ns + L - 1
    out = torch.empty(nout, dtype=torch.complex64, device="cuda")
    _, pk = xc(torch.from_numpy(s).cuda(), mode, out=out)
    r, _ = ref.cross_correlate_signals(pre, s, mode)
    c = out.cpu().numpy()
    assert np.abs(c - r).max() <= 1e-5 * np.abs(r).max()
    peak, idx, s1, s2 = gpu.dsp._read_peak(pk)
    a = np.abs(r)
    assert idx == int(np.argmax(a))
    assert peak == a.max()
    assert s1 == pytest.approx(a.sum(), rel=1e-5)


@pytest.mark.parametrize("dt", [np.complex64, np.complex128, np.float64])
def test_input_dtypes(gpu, dt):
    """complex64 operands refine in complex64 values (exact upcast); complex128
    and real float64 ones keep their 64-bit values for the refine pass."""
    rng = np.random.default_rng(3)
    if dt == np.float64:
        s = rng.standard_normal(40_000)
        t = s[12_000:12_400].copy()
    else:
        s = (rng.standard_normal(40_000) + 1j * rng.standard_normal(40_000)).astype(dt)
        t = s[12_000:12_400].copy()
    want = ref.find_correlation_peak(*ref.cross_correlate_signals(t, s, "full"))
    got = gpu.correlate_peak(t, s, "full")
    assert got[0] == want[0]
    assert got[1] == want[1]
    c, lags = gpu.cross_correlate_signals(t, s, "full")
    assert c.dtype == np.complex128
    assert gpu.find_correlation_peak(c, lags)[0] == want[0]


@pytest.mark.parametrize("L", [700, 2048, 4096, 8000, 12_000])
@pytest.mark.parametrize("ratio", [1 + 1e-9, 1 - 1e-9])
@pytest.mark.parametrize("swapped", [False, True])
def test_near_tie_columns_every_plan(gpu, L, ratio, swapped):
    """Two copies 1e-9 apart in amplitude whose peaks lie L + 197 outputs
    apart (other thread columns, where the correlator writes lane keys: M =
    16384 / 32768; whole waves at M = 4096 / 8192), in both operand orders
    (swapped: the template is the first operand, the kernel's outputs
    reversed): numpy's lag exactly, the peak to 1e-12."""
    n = 3 * L + 40_000
    pre = ref.qpsk_preamble(L, seed=L + 1)
    s = np.zeros(n, np.complex128)
    s[: n // 4] = 0.01 * ref.synth_iq(n // 4, seed=L)
    k1 = n // 3
    k2 = k1 + L + 197
    s[k1:k1 + L] += pre
    s[k2:k2 + L] += ratio * pre.astype(np.complex128)
    a, b = (s, pre) if swapped else (pre, s)
    mode = "full" if swapped else "valid"
    want = ref.find_correlation_peak(*ref.cross_correlate_signals(a, b, mode))
    lag, val, _ = gpu.correlate_peak(a, b, mode)
    assert lag == want[0]
    assert val == want[1]
    assert _status(gpu)[0] == 0


def test_flat_correlation_2e24_dense(gpu):
    """A tone against itself over 2^24 samples, 'valid' (M = 16384, 5461 blocks):
    every one of the 2^24 - 4095 outputs is a candidate.  No cap: the dense form
    evaluates all of them in numpy's order (status 0); the record's |c| is
    numpy's value at the returned lag (oracle/npdot.c), and the pass costs
    milliseconds (numpy: about half a minute)."""
    import time
    import torch
    from oracle import npdot
    n, L = 1 << 24, 4096
    ph = 2 * np.pi * 0.01 * np.arange(n)
    tone = torch.polar(torch.ones(n, dtype=torch.float64),
                       torch.from_numpy(ph)).to(torch.complex64).cuda()
    tmpl = tone[:L].cpu().numpy()
    gpu.correlate_peak(tmpl, tone, "valid")           # warm-up (plans, scratch)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    lag, val, _ = gpu.correlate_peak(tmpl, tone, "valid")
    dt = time.perf_counter() - t0
    st, cand = _status(gpu)
    print(f"2^24 flat: {cand} candidate items, {dt * 1e3:.1f} ms")
    assert st == 0 and cand > (1 << 20) // 64
    assert 0 <= lag < n - L + 1
    seg = tone[int(lag):int(lag) + L].cpu().numpy().astype(np.complex128)
    want = npdot.cabs(np.array([npdot.zdotu(seg, np.conj(tmpl.astype(np.complex128)), 1)]))[0]
    assert val == want
    assert dt < 0.5


def _set_watchdog(gpu, us):
    ctx = gpu.get_context()
    ctx.check(ctx.lib.vsig_set_option(ctx.h, b"refine_watchdog_us", int(us)), "watchdog")


def test_watchdog_fire_is_an_error_and_recovers(gpu):
    """A refine whose watchdog fires (forced: a 1 us bound, shorter than the
    finalize takes to publish the keys) is an error on every product path --
    the numpy front end, the sharded StreamChain (its gathered row is poisoned
    too) and the native chain -- never a warning; vsig_refine_status reports it
    once and clears the one-launch refine's counters, so the next correlation
    with the default bound gives numpy's lag and |c| exactly again (ADVICE r04:
    a fire must not leave stale counters behind)."""
    from vector_amd.shard import ChainConfig, HipBackend, NativeChain, StreamChain
    L, n, k0 = 4096, 1 << 20, 333_333
    pre = ref.qpsk_preamble(L, seed=5)
    s = ref.synth_iq(n, seed=6)
    s[k0:k0 + L] += pre
    want = ref.xcorr_peak(s, pre, "valid")
    assert want[1] == k0
    ctx = gpu.get_context()
    import ctypes as C
    v = C.c_int()
    ctx.check(ctx.lib.vsig_get_option(ctx.h, b"refine_watchdog_us", C.byref(v)), "get")
    assert v.value == 2_000_000
    # 1. numpy front end
    _set_watchdog(gpu, 1)
    try:
        with pytest.raises(gpu.RefineFault):
            gpu.correlate_peak(pre, s, "valid")
        assert _status(gpu)[0] == 2              # reported once; the counters are clear
    finally:
        _set_watchdog(gpu, 2_000_000)
    for _ in range(3):                           # clean launches again, exact each time
        lag, val, _ = gpu.correlate_peak(pre, s, "valid")
        assert (lag, val) == (want[1], want[2])
        assert _status(gpu)[0] == 0
    # 2. the sharded chain's classes (bench.py's path): global_peak raises
    taps = np.hanning(63).astype(np.float32)
    taps /= taps.sum()
    tmpl = pre[:1024].copy()
    cfg = ChainConfig(n_local=n, taps=taps, decim=1, nfft=1024, template=tmpl)
    ch = StreamChain(cfg, HipBackend(cfg, 0), 0, 1)
    ch.x.copy_(torch.from_numpy(s).cuda())
    _set_watchdog(gpu, 1)
    try:
        ch.step()
        with pytest.raises(gpu.RefineFault):
            ch.global_peak()
    finally:
        _set_watchdog(gpu, 2_000_000)
    ch.step()
    m, lag, _, _, _ = ch.global_peak()
    assert lag >= 0 and _status(gpu)[0] == 0
    ref_lag = lag
    # 3. the native chain (vsig_chain_result returns VSIG_E_REFINE)
    nat = NativeChain(cfg, 0)
    nat.load(torch.from_numpy(s).cuda())
    _set_watchdog(gpu, 1)
    try:
        nat.step()
        with pytest.raises(gpu.RefineFault):
            nat.global_peak()
    finally:
        _set_watchdog(gpu, 2_000_000)
    nat.step()
    assert nat.global_peak()[1] == ref_lag


def test_watchdog_fire_survives_scratch_growth(gpu):
    """a fire in a device-tensor Correlator pass whose
    status nobody read lives in the refine scratch's sticky fault word; when
    the next, larger correlation grows that scratch the fault is carried into
    the new one, so vsig_refine_status still reports 3 ('fired in some pass
    since the last call'), and the pass after the report is clean and exact.
    Runs on a fresh thread: its own context, so the scratch starts small."""
    import threading
    L, k1 = 4096, 5_000_011
    pre = ref.qpsk_preamble(L, seed=5)
    small = ref.synth_iq(1 << 20, seed=6)
    big = ref.synth_iq(1 << 23, seed=7)
    big[k1:k1 + L] += pre
    res = {}

    def body():
        try:
            xc = gpu.dsp.Correlator(pre)            # this thread's own context
            ctx = xc.ctx

            def wd(us):
                ctx.check(ctx.lib.vsig_set_option(ctx.h, b"refine_watchdog_us", int(us)), "wd")
            ds, db = torch.from_numpy(small).cuda(), torch.from_numpy(big).cuda()
            wd(1)
            try:
                xc(ds, "valid")                     # fires; nothing reads the status here
                torch.cuda.synchronize()
            finally:
                wd(2_000_000)
            xc(db, "valid")                          # 8x the partials: a larger scratch
            torch.cuda.synchronize()
            res["after_growth"] = gpu.dsp.refine_status(ctx)[0]
            _, pk = xc(db, "valid")
            res["peak"] = gpu.dsp._read_peak(pk)
            res["clean"] = gpu.dsp.refine_status(ctx)[0]
        except BaseException as e:                   # re-raised in the test's thread
            res["err"] = e

    th = threading.Thread(target=body)
    th.start()
    th.join()
    if "err" in res:
        raise res["err"]
    assert res["after_growth"] == 3
    assert res["clean"] == 0
    assert res["peak"][1] == k1


@pytest.mark.parametrize("snr_db", [60, 40, 30, 20, 10, 0])
def test_tone_under_noise_confidence(gpu, snr_db):
    """A tone template over a tone under complex noise: |c| has a high mean and
    a spread from rounding-noise-flat (60 dB) to Rayleigh-like (0 dB), across
    the fused sums' cancellation floor (dsp._FUSED_VAR_FLOOR).  Lag and |c|
    exactly numpy's, the confidence (utils.py:1328-1340) within 1e-5 on both
    sides of the floor (tone plus weak noise)."""
    n, L = 60_000, 2000
    t = np.arange(n)
    rng = np.random.default_rng(snr_db + 100)
    tone = np.exp(2j * np.pi * 0.0173 * t)
    sig = 10 ** (-snr_db / 20.0)
    x = (tone + sig * (rng.standard_normal(n) + 1j * rng.standard_normal(n)) / np.sqrt(2)).astype(np.complex64)
    tm = tone[:L].astype(np.complex64)
    want = ref.find_correlation_peak(*ref.cross_correlate_signals(tm, x, "valid"))
    lag, val, conf = gpu.correlate_peak(tm, x, "valid")
    assert _status(gpu)[0] == 0
    assert lag == want[0]
    assert val == want[1]
    assert conf == pytest.approx(want[2], rel=1e-5, abs=1e-7)
