"""Pin the CPU oracle (oracle/ref.py) against the reference's own outputs
(tests/golden/*.npz, produced by tests/golden/make_golden.py from the
reference's utils.py) and the reference tests' known answers.  CPU only."""
import glob
import os

import numpy as np
import pytest

from conftest import GOLDEN, golden
from oracle import ref


def test_spectrogram_params_table():
    g = golden("spec_params.npz")
    cols = list(g["columns"])
    for row in g["table"]:
        r = dict(zip(cols, row))
        p = ref.spectrogram_params(int(r["n"]), r["sr"], int(r["max_samples"]),
                                   r["time_res_us"], bool(r["adaptive"]))
        assert p["nsig"] == r["nsig"]
        assert p["fs"] == pytest.approx(r["fs"], rel=1e-15)
        assert (p["nperseg"], p["noverlap"], p["nfft"]) == (r["nperseg"], r["noverlap"], r["nfft"])
        assert (p["window"] == "hann") == bool(r["window_is_hann"])


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "spec_*.npz"))))
def test_create_spectrogram_outputs(path):
    if path.endswith("spec_params.npz"):
        pytest.skip("parameter table")
    g = np.load(path)
    f, t, S = ref.create_spectrogram(g["x"], float(g["sr"]))
    assert tuple(S.shape) == tuple(g["shape"])
    np.testing.assert_array_equal(f, g["f"])
    np.testing.assert_array_equal(t, g["t"])
    np.testing.assert_array_equal(S[:, g["sel"]], g["Sxx_sel"])
    np.testing.assert_allclose(S.astype(np.float64).sum(axis=0), g["frame_sum"], rtol=1e-12)


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "stft_*.npz"))))
def test_stft_outputs(path):
    g = np.load(path)
    f, t, S = ref.spectrum(g["x"], 56e6, str(g["window"]), int(g["nperseg"]),
                           int(g["noverlap"]), int(g["nfft"]))
    np.testing.assert_array_equal(S, g["Sxx"])
    np.testing.assert_array_equal(f, g["f"])
    np.testing.assert_array_equal(t, g["t"])


def test_cross_correlate_small():
    g = golden("xcorr_small.npz")
    for mode in ("full", "valid", "same"):
        c, lags = ref.cross_correlate_signals(g["s1"], g["s2"], mode)
        np.testing.assert_array_equal(c, g[f"c_{mode}"])
        np.testing.assert_array_equal(lags, g[f"lags_{mode}"])
        if f"peak_{mode}" in g:
            lag, val, conf = ref.find_correlation_peak(c, lags)
            np.testing.assert_allclose([lag, val, conf], g[f"peak_{mode}"], rtol=1e-12)
        else:
            with pytest.raises(IndexError):
                ref.find_correlation_peak(c, lags)
    c, lags = ref.cross_correlate_signals(g["s1"], g["s1"])
    np.testing.assert_allclose(ref.find_correlation_peak(c, lags), g["self_peak"], rtol=1e-12)
    # test_packet_transplant.py:40-68 known answers
    assert len(c) == 2 * len(g["s1"]) - 1 and c.dtype == np.complex128
    assert ref.find_correlation_peak(c, lags)[0] == 0


def test_xcorr_peak_4096():
    g = golden("xcorr_peak.npz")
    i, lag, peak, s1, s2, conf = ref.xcorr_peak(g["x"], g["pre"], "valid")
    assert lag == int(g["peak_lag"]) == int(g["k0"])
    assert peak == pytest.approx(float(g["peak_val"]), rel=1e-12)
    assert conf == pytest.approx(float(g["conf"]), abs=1e-12)
    assert s1 == pytest.approx(float(g["sum_abs"]), rel=1e-12)
    assert s2 == pytest.approx(float(g["sum_abs2"]), rel=1e-12)


def test_packet_functions():
    g = golden("packet.npz")
    sig = np.concatenate([np.zeros(100), np.ones(50), np.zeros(20)])
    assert ref.find_packet_start(sig) == int(g["energy_start"])
    assert 98 <= ref.find_packet_start(sig) <= 102                    # tests/test_utils.py:24-27
    tm = np.array([1.0, 1.0, 1.0])
    sig2 = np.concatenate([np.zeros(10), tm, np.zeros(5)])
    assert ref.find_packet_start(sig2, template=tm) == int(g["template_start"]) == 10  # :30-34
    x = g["burst_x"]
    assert ref.find_packet_start(x) == int(g["burst_start"])
    np.testing.assert_array_equal(ref.detect_packet_bounds(x, 56e6), g["burst_bounds"])
    assert ref.find_packet_start(x[:80_000], template=x[61_234:61_234 + 512]) == int(g["burst_template_start"])
    np.testing.assert_allclose(ref.find_packet_location_in_vector(g["loc_vector"], g["loc_packet"], g["loc_ref"]),
                               g["loc_result"], rtol=1e-12)
    np.testing.assert_allclose(ref.find_packet_location_in_vector(
        g["loc_vector"], g["loc_packet"], g["loc_ref"], search_window=(10_000, 20_000)),
        g["loc_result_win"], rtol=1e-12)


def test_fir_numpy_semantics():
    g = golden("fir.npz")
    for nt in (63, 255):
        for d in (1, 4):
            np.testing.assert_array_equal(ref.fir_filter(g["x"], g[f"taps{nt}"], d), g[f"y{nt}_d{d}"])


def test_pfb_definition_small():
    # direct double loop of the definition in ref.pfb_channelize's docstring
    rng = np.random.default_rng(0)
    C, P = 8, 4
    h = rng.standard_normal(C * P)
    x = (rng.standard_normal(200) + 1j * rng.standard_normal(200)).astype(np.complex64)
    y = ref.pfb_channelize(x, h, C)
    M = (len(x) - P * C) // C + 1
    assert y.shape == (C, M)
    for m in (0, 3, M - 1):
        z = np.array([sum(h[q * C + p] * x[m * C + q * C + p] for q in range(P)) for p in range(C)])
        for k in range(C):
            want = sum(z[p] * np.exp(-2j * np.pi * k * p / C) for p in range(C))
            assert abs(y[k, m] - want) < 1e-4 * (1 + abs(want))


def test_synthetic_generators_deterministic():
    a = ref.synth_iq(1000, seed=3)
    b = ref.synth_iq(1000, seed=3)
    np.testing.assert_array_equal(a, b)
    p = ref.qpsk_preamble(64)
    np.testing.assert_allclose(np.abs(p), 1.0, rtol=1e-6)


# ---------------------------------------------------------------- round-2 fixtures
def test_tone_transplant_oracle():
    """The reference's own tone data (data/packet_*.mat in data/fixed_test_vector.mat):
    the oracle's argmax, peak and confidence equal the reference's bit for bit."""
    g = golden("tone_transplant.npz")
    vec = g["vector"]
    for i in range(1, 7):
        seg = g[f"seg{i}"]
        c, lags = ref.cross_correlate_signals(seg, vec)
        assert int(np.argmax(np.abs(c))) == int(g[f"vec{i}_argmax"])
        np.testing.assert_array_equal(np.array(ref.find_correlation_peak(c, lags), np.float64),
                                      g[f"vec{i}_peak"])
    for i in (1, 3):
        pk, seg = g[f"packet{i}"], g[f"seg{i}"]
        c, lags = ref.cross_correlate_signals(seg, pk)
        assert int(np.argmax(np.abs(c))) == int(g[f"pkt{i}_argmax"])
        np.testing.assert_array_equal(
            np.array(ref.find_packet_location_in_vector(vec, pk, seg), np.float64), g[f"loc{i}"])


def test_stream_ops_oracle():
    g = golden("stream_ops.npz")
    x = g["shift_x"]
    for j in range(3):
        f, sr = g[f"shift{j}_args"]
        np.testing.assert_array_equal(ref.apply_frequency_shift(x, f, sr), g[f"shift{j}"])
    for j in range(4):
        vl, pl, rl, npow = (int(v) for v in g[f"tp{j}_args"])
        out = ref.transplant_packet_in_vector(g["tp_vector"], g["tp_packet"], vl, pl,
                                              None if rl < 0 else rl, bool(npow))
        np.testing.assert_array_equal(out, g[f"tp{j}"])
    for j in range(5):
        a, b = g[f"rs{j}_sr"]
        y = ref.resample_signal(g[f"rs{j}_x"], a, b)
        assert y.dtype == np.complex64 and y.shape == g[f"rs{j}"].shape
        np.testing.assert_array_equal(y, g[f"rs{j}"])


def test_wv_oracle():
    """mat2wv's payload and level fields from the oracle against the bytes of the
    file the reference wrote (everything but its DATE field)."""
    g = golden("wv.npz")
    for j in range(3):
        sr, norm = g[f"args{j}"]
        raw = g[f"bytes{j}"].tobytes()
        payload, rms, peak = ref.mat2wv_fields(g[f"x{j}"], bool(norm))
        head = raw[: raw.index(b"#") + 1]
        assert raw[len(head):] == payload.tobytes() + b"}"
        assert f"{{LEVEL OFFS: {rms}, {peak}}}".encode() in head
        assert f"{{CLOCK: {sr}}}".encode() in head
        assert f"{{SAMPLES: {len(g[f'x{j}'])}}}".encode() in head


def test_channel_oracle():
    g = golden("channel.npz")
    for j in range(5):
        cf, sr, bw = g[f"args{j}"]
        np.testing.assert_array_equal(ref.filter_channel(g[f"x{j}"], cf, sr, bw), g[f"y{j}"])
    assert str(g["odd_raises"]) == "ValueError"
    with pytest.raises(ValueError):
        ref.filter_channel(ref.synth_iq(1001, seed=45), 5220e6, 56e6, 20e6)
