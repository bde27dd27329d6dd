"""Host-side logic of the analysis front end (vector_amd/analysis.py) on CPU:
numpy's percentile / median rules restated over order statistics must give
numpy's exact numbers and dtypes (the GPU only supplies the k-th smallest
values, which are exact), and the oracle's detection helpers must reproduce
the reference's known answers (tests/test_utils.py of the reference)."""
import numpy as np
import pytest

from conftest import golden
from oracle import ref
from vector_amd.analysis import _median, _percentile


@pytest.mark.parametrize("dt", [np.float32, np.float64])
def test_percentile_restatement_is_bit_exact(dt):
    rng = np.random.default_rng(7)
    for trial in range(400):
        n = int(rng.integers(1, 40)) if trial < 300 else int(rng.integers(1, 5000))
        a = (rng.standard_normal(n) * 10 ** rng.uniform(-6, 6)).astype(dt)
        if trial % 5 == 0:
            a = np.round(a)                       # ties
        s = np.sort(a)

        def fetch(rk):
            return {r: s[r] for r in rk}
        for p in (0, 5, 10, 50, 95, 100, 12.345, float(rng.uniform(0, 100))):
            r, e = _percentile(n, p, dt, fetch), np.percentile(a, p)
            assert r == e and type(r) is type(e), (n, p, r, e)
        assert _median(n, dt, fetch) == np.median(a)


def test_percentile_rejects_out_of_range():
    with pytest.raises(ValueError):
        _percentile(10, 101, np.float64, lambda rk: {r: 0.0 for r in rk})


def test_median_empty_is_nan():
    assert np.isnan(_median(0, np.float64, lambda rk: {}))


def test_oracle_packet_known_answers():
    # reference tests/test_utils.py:24-34
    sig = np.concatenate([np.zeros(100), np.ones(50), np.zeros(20)])
    assert 98 <= ref.find_packet_start(sig) <= 102
    tmpl = np.array([1.0, 1.0, 1.0])
    assert ref.find_packet_start(np.concatenate([np.zeros(10), tmpl, np.zeros(5)]), template=tmpl) == 10
    g = golden("packet.npz")
    assert ref.find_packet_start(g["burst_x"]) == int(g["burst_start"])
    assert tuple(ref.detect_packet_bounds(g["burst_x"], 56e6)) == tuple(g["burst_bounds"])


def test_oracle_normalize_matches_numpy_restatement():
    rng = np.random.default_rng(1)
    S = (rng.exponential(size=(64, 40)) ** 3).astype(np.float32)
    S[::7] = 0
    db, vmin, vmax = ref.normalize_spectrogram(S)
    assert db.dtype == np.float32 and db.shape == S.shape
    assert vmax - vmin <= 25 + 1e-4
