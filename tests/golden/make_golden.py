"""Generate the golden fixtures in tests/golden/ from the REFERENCE itself.

Run in the build container only (needs /root/reference, read-only):

    PYTHONDONTWRITEBYTECODE=1 MPLBACKEND=Agg python tests/golden/make_golden.py

It imports the reference's ``utils`` module (ramiyako/vector ``utils.py``) and
records inputs + outputs of the hot-path functions as small ``.npz`` files.
Nothing from the reference's source is copied; only data (inputs, outputs,
parameters) is stored.  The GPU box never runs this script.

Fixture inventory (SURVEY.md §8(c) golden set G1-G5):
  spec_params.npz      create_spectrogram parameter logic (utils.py:161-276)
                       recorded from the reference's own scipy call, N up to 2**28
  spec_<case>.npz      create_spectrogram(sig, sr) outputs (f, t, Sxx) for small inputs
                       incl. the reference's real data files (data/*.mat, sample_vector.mat)
  stft_<case>.npz      the scipy.signal.spectrogram call the reference makes
                       (utils.py:281-291) at BASELINE C1/C2 shapes (reduced N)
  xcorr_small.npz      cross_correlate_signals full/valid/same arrays (utils.py:1258-1295)
                       + find_correlation_peak (utils.py:1298-1342)
  xcorr_peak.npz       L=4096 QPSK preamble in a 2**17 stream: peak lag/value/confidence
  packet.npz           find_packet_start / detect_packet_bounds /
                       find_packet_location_in_vector results (utils.py:784-825, 1372-1434)
  fir.npz              np.convolve(x, taps)[:N][::D] (no reference FIR: numpy-pinned)
  tone_transplant.npz  the reference's own tone data (data/fixed_test_vector.mat and
                       data/packet_{1..6}.mat): cross_correlate_signals +
                       find_correlation_peak of each packet's first 4096 samples in the
                       vector (full mode) and, for packets 1 and 3, in their own packet and
                       find_packet_location_in_vector (utils.py:1258-1342, 1372-1434) --
                       near-tie argmaxes (top-2 |c| gaps 1e-13 .. 7e-12 relative)
  refine_flat.npz      flat |c| (every full-overlap output an exact tie): a 2^21-sample
                       tone against its first 4096 samples, 30 periods of
                       data/packet_1.mat in a vector, a tone template over a tone
                       ('valid', numpy's confidence from a rounding-noise std)
  stream_ops.npz       apply_frequency_shift (utils.py:120-127), transplant_packet_in_vector
                       (utils.py:1437-1501), resample_signal (utils.py:107-118)
  wv.npz               mat2wv's SMU-WV file bytes (vector_analyzer/mat_to_wv_converter.py:7-64)
                       for a synthetic and the reference's sample_vector.mat, normalised or not
  channel.npz          filter_channel (vector_analyzer/split_channels.py:15-44)
"""
from __future__ import annotations

import os
import sys

import numpy as np
import scipy
import scipy.io as sio
import scipy.signal

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
sys.path.insert(0, os.path.join(HERE, "..", ".."))
sys.path.insert(0, REF)

import utils as refutils  # noqa: E402  (the reference)

from oracle.ref import qpsk_preamble, synth_iq  # noqa: E402  (seeded generators only)

META = dict(numpy=np.__version__, scipy=scipy.__version__,
            reference="ramiyako/vector@2025-07-18 utils.py")


def save(name, **arrs):
    arrs.update({f"meta_{k}": np.array(v) for k, v in META.items()})
    np.savez_compressed(os.path.join(HERE, name), **arrs)
    print("wrote", name, {k: getattr(v, "shape", None) for k, v in arrs.items()
                          if not k.startswith("meta_")})


class Recorder:
    """Wraps scipy.signal.spectrogram inside the reference module to record the
    exact arguments create_spectrogram passes (optionally skipping the call)."""

    def __init__(self, dry=False):
        self.calls = []
        self.dry = dry
        self.real = scipy.signal.spectrogram

    def __call__(self, x, fs=1.0, window="hann", nperseg=None, noverlap=None,
                 nfft=None, **kw):
        self.calls.append(dict(n=len(x), fs=fs, window=window, nperseg=nperseg,
                               noverlap=noverlap, nfft=nfft, kw=kw))
        if self.dry:
            nfr = max(1, (len(x) - nperseg) // (nperseg - noverlap) + 1)
            return (np.fft.fftfreq(nfft, 1 / fs), np.arange(nfr, dtype=float),
                    np.ones((nfft, nfr), np.float32))
        return self.real(x, fs=fs, window=window, nperseg=nperseg,
                         noverlap=noverlap, nfft=nfft, **kw)


def record_spectrogram(sig, sr, dry=False, **kw):
    rec = Recorder(dry)
    orig = refutils.scipy.signal.spectrogram
    refutils.scipy.signal.spectrogram = rec
    try:
        out = refutils.create_spectrogram(sig, sr, **kw)
    finally:
        refutils.scipy.signal.spectrogram = orig
    return out, rec.calls


def gen_spec_params():
    cases = []
    for n in (500, 2_000, 10_000, 50_000, 140_000, 2 ** 16, 2 ** 20, 1_500_000,
              3_000_000, 10_000_000, 15_000_000, 2 ** 28):
        for sr in (56e6, 10e6, 8000.0):
            cases.append((n, sr, 2_000_000, 1, True))
    cases += [(10_000_000, 56e6, 1_000_000, 50, True), (2 ** 20, 56e6, 2_000_000, 1, False),
              (3_000_000, 56e6, 5_000_000, 10, True), (500_000, 56e6, 2_000_000, 25, True)]
    rows = []
    for n, sr, ms, tr, ad in cases:
        sig = np.broadcast_to(np.complex64(1 + 1j), (n,))
        (_, _, _), calls = record_spectrogram(sig, sr, dry=True, max_samples=ms,
                                              time_resolution_us=tr,
                                              adaptive_resolution=ad)
        c = calls[0]
        rows.append((n, sr, ms, tr, int(ad), c["n"], c["fs"], c["nperseg"],
                     c["noverlap"], c["nfft"], 1 if c["window"] == "hann" else 0))
    a = np.array(rows, dtype=np.float64)
    save("spec_params.npz", table=a,
         columns=np.array("n sr max_samples time_res_us adaptive nsig fs nperseg "
                          "noverlap nfft window_is_hann".split()))


def frame_subset(nframes, keep=96):
    """Frames stored in full (first, last, and evenly spaced); every frame's
    float64 sum is stored too, so the whole output is still checked."""
    if nframes <= keep:
        return np.arange(nframes)
    return np.unique(np.concatenate([np.arange(8), np.arange(nframes - 8, nframes),
                                     np.linspace(0, nframes - 1, keep - 16).astype(int)]))


def gen_spec_outputs():
    cases = {}
    cases["synth16k_56M"] = (synth_iq(16384, seed=1), 56e6)
    cases["synth64k_56M"] = (synth_iq(2 ** 16, seed=2), 56e6)
    cases["tone_8k"] = (refutils.apply_frequency_shift(
        refutils.generate_sample_packet(0.1, 8000, 1000), 500, 8000), 8000.0)
    sv = sio.loadmat(os.path.join(REF, "sample_vector.mat"), squeeze_me=True)["Y"]
    cases["sample_vector_56M"] = (np.asarray(sv).ravel().astype(np.complex64), 56e6)
    pk = sio.loadmat(os.path.join(REF, "data", "packet_3_bpsk.mat"), squeeze_me=True)["Y"]
    cases["packet3_bpsk_56M"] = (np.asarray(pk).ravel().astype(np.complex64), 56e6)
    cases["sparse_zeros"] = (np.zeros(4096, np.complex64), 56e6)
    for name, (sig, sr) in cases.items():
        (f, t, S), calls = record_spectrogram(sig, sr)
        c = calls[-1]
        S = S.astype(np.float32)
        sel = frame_subset(S.shape[1])
        save(f"spec_{name}.npz", x=sig, sr=np.float64(sr), f=f, t=t,
             Sxx_sel=S[:, sel], sel=sel, frame_sum=S.astype(np.float64).sum(axis=0),
             shape=np.array(S.shape), nperseg=c["nperseg"], noverlap=c["noverlap"],
             nfft=c["nfft"], window=np.array(c["window"]), ncalls=len(calls))


def gen_stft():
    # BASELINE C1 shape (reduced N) and C2 shape (reduced N), exactly the kwargs
    # the reference passes at utils.py:281-291.
    for name, n, win, nps, nov, nfft in (("c1_1024", 2 ** 16, "hann", 1024, 0, 1024),
                                         ("c2_8192", 2 ** 17, "hann", 8192, 0, 8192),
                                         ("bh_ovl", 2 ** 15, "blackmanharris", 1000, 900, 2048),
                                         ("box_small", 3000, "boxcar", 32, 16, 64)):
        x = synth_iq(n, seed=n + nps)
        f, t, S = scipy.signal.spectrogram(x, fs=56e6, window=win, nperseg=nps,
                                           noverlap=nov, nfft=nfft,
                                           return_onesided=False, detrend=False,
                                           scaling="spectrum")
        save(f"stft_{name}.npz", x=x, f=f, t=t, Sxx=S.astype(np.float32),
             nperseg=nps, noverlap=nov, nfft=nfft, window=np.array(win))


def gen_xcorr():
    rng = np.random.default_rng(7)
    s1 = (rng.standard_normal(64) + 1j * rng.standard_normal(64)).astype(np.complex64)
    s2 = (rng.standard_normal(2048) + 1j * rng.standard_normal(2048)).astype(np.complex64)
    s2[700:764] += 3 * s1
    out = dict(s1=s1, s2=s2)
    for mode in ("full", "valid", "same"):
        c, lags = refutils.cross_correlate_signals(s1, s2, mode=mode)
        out[f"c_{mode}"] = c
        out[f"lags_{mode}"] = lags
        try:
            lag, val, conf = refutils.find_correlation_peak(c, lags)
            out[f"peak_{mode}"] = np.array([lag, val, conf], np.float64)
        except IndexError:
            # 'same' mode: len(lags) = L + L%2 != len(c) (utils.py:1290-1291), so
            # the reference's find_correlation_peak raises IndexError whenever the
            # argmax lies beyond len(lags).  Recorded as behaviour to reproduce.
            out[f"peak_{mode}_raises"] = np.array("IndexError")
    # zero-lag identity case (test_packet_transplant.py:57-68)
    c, lags = refutils.cross_correlate_signals(s1, s1)
    out["self_peak"] = np.array(refutils.find_correlation_peak(c, lags), np.float64)
    save("xcorr_small.npz", **out)

    L, n, k0 = 4096, 2 ** 17, 100_003
    pre = qpsk_preamble(L)
    x = synth_iq(n, seed=11)
    x[k0:k0 + L] += pre
    c, lags = refutils.cross_correlate_signals(pre, x, mode="valid")
    a = np.abs(c)
    lag, val, conf = refutils.find_correlation_peak(c, lags)
    save("xcorr_peak.npz", x=x, pre=pre, k0=k0, peak_lag=lag, peak_val=val,
         conf=conf, sum_abs=a.sum(), sum_abs2=(a * a).sum(),
         top2=np.sort(a)[-2:])
    c, lags = refutils.cross_correlate_signals(pre, x, mode="full")
    lag, val, conf = refutils.find_correlation_peak(c, lags)
    save("xcorr_peak_full.npz", peak_lag=lag, peak_val=val, conf=conf)


def gen_packet():
    out = {}
    # reference tests' known answers (tests/test_utils.py:24-34)
    sig = np.concatenate([np.zeros(100), np.ones(50), np.zeros(20)])
    out["energy_start"] = refutils.find_packet_start(sig)
    tmpl = np.array([1.0, 1.0, 1.0])
    sig2 = np.concatenate([np.zeros(10), tmpl, np.zeros(5)])
    out["template_start"] = refutils.find_packet_start(sig2, template=tmpl)
    # synthetic burst
    rng = np.random.default_rng(3)
    n = 200_000
    x = (0.01 * (rng.standard_normal(n) + 1j * rng.standard_normal(n))).astype(np.complex64)
    x[61_234:141_000] += np.exp(2j * np.pi * 0.013 * np.arange(141_000 - 61_234))
    out["burst_x"] = x
    out["burst_start"] = refutils.find_packet_start(x)
    out["burst_bounds"] = np.array(refutils.detect_packet_bounds(x, 56e6))
    tm = x[61_234:61_234 + 512].copy()
    out["burst_template_start"] = refutils.find_packet_start(x[:80_000], template=tm)
    # transplant localisation with a unique-peak QPSK reference
    ref = qpsk_preamble(256, seed=99)
    packet = (0.05 * (rng.standard_normal(4000) + 1j * rng.standard_normal(4000))).astype(np.complex64)
    packet[500:756] += ref
    vec = (0.05 * (rng.standard_normal(30000) + 1j * rng.standard_normal(30000))).astype(np.complex64)
    vec[12_345:12_601] += ref
    out["loc_ref"], out["loc_packet"], out["loc_vector"] = ref, packet, vec
    out["loc_result"] = np.array(refutils.find_packet_location_in_vector(vec, packet, ref), np.float64)
    out["loc_result_win"] = np.array(refutils.find_packet_location_in_vector(
        vec, packet, ref, search_window=(10_000, 20_000)), np.float64)
    save("packet.npz", **out)


def gen_fir():
    x = synth_iq(2 ** 16, seed=5)
    t63 = scipy.signal.firwin(63, 0.25).astype(np.float32)
    t255 = scipy.signal.firwin(255, 0.2).astype(np.float32)
    out = dict(x=x, taps63=t63, taps255=t255)
    for nt, t in ((63, t63), (255, t255)):
        for d in (1, 4):
            out[f"y{nt}_d{d}"] = np.convolve(x, t, mode="full")[: len(x)][::d]
    save("fir.npz", **out)


def gen_tone_transplant():
    """The transplant workflow on the reference's own data (unified_gui.py:1105-1131:
    reference segment = a slice of the packet, located in the vector and in the
    packet).  Packets are complex128 (the .mat files' own precision), the
    vector complex64."""
    vec = np.asarray(sio.loadmat(os.path.join(REF, "data", "fixed_test_vector.mat"))["Y"]).ravel()
    out = dict(vector=vec)
    for i in range(1, 7):
        pk = np.asarray(sio.loadmat(os.path.join(REF, "data", f"packet_{i}.mat"))["Y"]).ravel()
        seg = refutils.extract_reference_segment(pk, 0, 4096)
        out[f"seg{i}"] = seg
        c, lags = refutils.cross_correlate_signals(seg, vec)
        lag, val, conf = refutils.find_correlation_peak(c, lags)
        a = np.abs(c)
        top = np.argsort(a)[::-1][:8]
        out[f"vec{i}_peak"] = np.array([lag, val, conf], np.float64)
        out[f"vec{i}_argmax"] = np.int64(np.argmax(a))
        out[f"vec{i}_top_idx"] = top
        out[f"vec{i}_top_abs"] = a[top]
        out[f"vec{i}_sums"] = np.array([a.sum(), (a * a).sum()])
        if i in (1, 3):
            out[f"packet{i}"] = pk
            c, lags = refutils.cross_correlate_signals(seg, pk)
            a = np.abs(c)
            out[f"pkt{i}_peak"] = np.array(refutils.find_correlation_peak(c, lags), np.float64)
            out[f"pkt{i}_argmax"] = np.int64(np.argmax(a))
            out[f"pkt{i}_nearmax"] = np.int64(np.count_nonzero(a >= a.max() * (1 - 1e-12)))
            out[f"loc{i}"] = np.array(refutils.find_packet_location_in_vector(vec, pk, seg),
                                      np.float64)
    save("tone_transplant.npz", **out)


def gen_refine_flat():
    """Flat |c| on the reference's own kind of data, where every full-overlap
    output ties with the maximum up to numpy's rounding (np.argmax's pick and
    np.std are decided by the rounding of numpy's own sums):
      (a) a 2^21-sample tone (generate_sample_packet, utils.py:679-686) against
          its first 4096 samples, 'full' (cross_correlate_signals +
          find_correlation_peak, utils.py:1258-1342); the tone is regenerated
          by the tests (oracle.ref.generate_sample_packet) and checked against
          the sha256 stored here;
      (b) 30 instances of data/packet_1.mat (load_packet_info, complex64) in
          a vector built as unified_gui.py:1712, 1755-1769 does (period 56000
          samples), against seg1 = the .mat packet's first 4096 samples
          (complex128), and find_packet_location_in_vector;
      (c) a 1000-sample tone template over a 20000-sample tone, 'valid': every
          output in the band, numpy's std = rounding noise (confidence > 0)."""
    import hashlib
    from oracle.ref import periodic_vector
    out = {}
    # (a)
    dur, sr, f = 1.0, float(2 ** 21), 40_961.5
    tone = refutils.generate_sample_packet(dur, sr, f)
    seg = refutils.extract_reference_segment(tone, 0, 4096)
    c, lags = refutils.cross_correlate_signals(seg, tone)
    lag, val, conf = refutils.find_correlation_peak(c, lags)
    a = np.abs(c)
    out.update(a_args=np.array([dur, sr, f]), a_sha=np.array(hashlib.sha256(tone.tobytes()).hexdigest()),
               a_peak=np.array([lag, val, conf], np.float64), a_argmax=np.int64(np.argmax(a)),
               a_nearmax=np.int64(np.count_nonzero(a >= a.max() * (1 - 1e-12))),
               a_stats=np.array([a.mean(), a.std()]))
    del c, a
    # (b)
    y, _pre = refutils.load_packet_info(os.path.join(REF, "data", "packet_1.mat"))
    pk = np.asarray(sio.loadmat(os.path.join(REF, "data", "packet_1.mat"))["Y"]).ravel()
    seg1 = refutils.extract_reference_segment(pk, 0, 4096)
    period, reps = 56_000, 30
    vec = periodic_vector(y, period, period * (reps - 1) + len(y))
    c, lags = refutils.cross_correlate_signals(seg1, vec)
    lag, val, conf = refutils.find_correlation_peak(c, lags)
    a = np.abs(c)
    out.update(b_args=np.array([period, reps, period * (reps - 1) + len(y)]),
               b_sha=np.array(hashlib.sha256(vec.tobytes()).hexdigest()),
               b_peak=np.array([lag, val, conf], np.float64), b_argmax=np.int64(np.argmax(a)),
               b_nearmax=np.int64(np.count_nonzero(a >= a.max() * (1 - 1e-12))),
               b_loc=np.array(refutils.find_packet_location_in_vector(vec, pk, seg1), np.float64))
    del c, a
    # (c)
    tone = refutils.generate_sample_packet(0.02, 1e6, 12_345.0)
    tm = refutils.extract_reference_segment(tone, 0, 1000)
    c, lags = refutils.cross_correlate_signals(tm, tone, mode="valid")
    lag, val, conf = refutils.find_correlation_peak(c, lags)
    a = np.abs(c)
    out.update(c_tone=tone, c_peak=np.array([lag, val, conf], np.float64),
               c_stats=np.array([a.mean(), a.std()]), c_abs=a)
    save("refine_flat.npz", **out)


def gen_stream_ops():
    import contextlib
    import io
    out = {}
    x = synth_iq(20_000, seed=21)
    for j, (f, sr) in enumerate(((1e6, 56e6), (-13.37e6, 56e6), (0.25e6, 1e6))):
        out[f"shift{j}_args"] = np.array([f, sr])
        out[f"shift{j}"] = refutils.apply_frequency_shift(x, f, sr)
    out["shift_x"] = x
    # transplant_packet_in_vector: the reference's real packet into a synthetic vector
    pk = np.asarray(sio.loadmat(os.path.join(REF, "data", "packet_3_bpsk.mat"))["Y"]).ravel()
    pk = pk[:6000].astype(np.complex64)
    vec = synth_iq(20_000, seed=22)
    out["tp_packet"], out["tp_vector"] = pk, vec
    cases = [dict(vector_location=1000), dict(vector_location=17_000),
             dict(vector_location=200, packet_location=100, replace_length=3000),
             dict(vector_location=5000, normalize_power=False)]
    for j, kw in enumerate(cases):
        with contextlib.redirect_stdout(io.StringIO()):
            out[f"tp{j}"] = refutils.transplant_packet_in_vector(vec, pk, **kw)
        out[f"tp{j}_args"] = np.array([kw.get("vector_location"), kw.get("packet_location", 0),
                                       kw.get("replace_length", -1),
                                       int(kw.get("normalize_power", True))])
    # resample_signal: scipy.signal.resample(x, int(len * ratio)).astype(complex64)
    rs = {"rs0": (synth_iq(10_000, seed=23), 56e6, 40e6), "rs1": (synth_iq(4096, seed=24), 10e6, 25e6),
          "rs2": (synth_iq(20_001, seed=25), 61.44e6, 56e6), "rs3": (pk[:4_321], 56e6, 56e6 * 1.5),
          "rs4": (synth_iq(1 << 15, seed=26), 56e6, 14e6)}
    for k, (sig, a, b) in rs.items():
        out[f"{k}_x"] = sig
        out[f"{k}_sr"] = np.array([a, b])
        out[k] = refutils.resample_signal(sig, a, b)
    save("stream_ops.npz", **out)


def gen_wv(tmpdir="/tmp"):
    import contextlib
    import io
    sys.path.insert(0, os.path.join(REF, "vector_analyzer"))
    import mat_to_wv_converter as m2w
    out = {}
    sv = np.asarray(sio.loadmat(os.path.join(REF, "sample_vector.mat"))["Y"]).ravel()
    for j, (sig, sr, norm) in enumerate(((synth_iq(3000, seed=31) * 0.3, 56e6, True),
                                         (synth_iq(3000, seed=32) * 0.3, 61.44e6, False),
                                         (sv, 56e6, True))):
        fn = os.path.join(tmpdir, f"golden_wv_{j}.wv")
        with contextlib.redirect_stdout(io.StringIO()):
            m2w.mat2wv(sig, fn, sr, bNormalize=norm)
        out[f"x{j}"] = sig
        out[f"args{j}"] = np.array([sr, int(norm)])
        out[f"bytes{j}"] = np.frombuffer(open(fn, "rb").read(), np.uint8)
        os.remove(fn)
    save("wv.npz", **out)


def gen_channel():
    sys.path.insert(0, os.path.join(REF, "vector_analyzer"))
    import split_channels as sc
    out = {}
    cases = [(synth_iq(1 << 14, seed=41), 5220e6, 56e6, 20e6),
             (synth_iq(12_000, seed=42), 5240e6, 56e6, 20e6),
             (synth_iq(4096, seed=43), 5230e6 - 300.0, 1000.0, 20e6),      # wide mask (small rate)
             (synth_iq(10_002, seed=44), 5230e6 + 2e6, 2000.0, 6e6)]
    pk = np.asarray(sio.loadmat(os.path.join(REF, "data", "packet_3_bpsk.mat"))["Y"]).ravel()
    cases.append((pk[:16_384], 5220e6, 56e6, 20e6))
    for j, (x, cf, sr, bw) in enumerate(cases):
        out[f"x{j}"] = x
        out[f"args{j}"] = np.array([cf, sr, bw])
        out[f"y{j}"] = sc.filter_channel(x, cf, sr, bw)
    try:
        sc.filter_channel(synth_iq(1001, seed=45), 5220e6, 56e6, 20e6)
        out["odd_raises"] = np.array("")
    except ValueError as e:
        out["odd_raises"] = np.array(type(e).__name__)
    save("channel.npz", **out)


if __name__ == "__main__":
    if len(sys.argv) > 1:
        for name in sys.argv[1:]:
            globals()[f"gen_{name}"]()
        sys.exit(0)
    gen_tone_transplant()
    gen_refine_flat()
    gen_stream_ops()
    gen_wv()
    gen_channel()
    gen_spec_params()
    gen_spec_outputs()
    gen_stft()
    gen_xcorr()
    gen_packet()
    gen_fir()
