"""The numpy-order restatement (oracle/npdot.c) against numpy itself, bit for
bit: np.dot / np.correlate over complex128 (OpenBLAS zdotu's accumulator
layout, tail and thread split) and np.abs on complex128 (numpy's SIMD formula,
which differs from hypot in a third of the cases).  refine.hip evaluates the
same order on the GPU; this pins what it must reproduce.  The reference's tone
self-correlations (tests/golden/tone_transplant.npz: exact ties in exact
arithmetic) are decided by exactly this order."""
import numpy as np
import pytest

from conftest import golden
from oracle import npdot, ref
from vector_amd._lib import numpy_blas_threads

T = numpy_blas_threads()


def _bits(x):
    return np.atleast_1d(np.asarray(x, np.complex128)).view(np.uint64)


def test_zdotu_every_length_class():
    rng = np.random.default_rng(1)
    lens = list(range(1, 70)) + [255, 256, 1000, 4095, 4096, 4097, 9999, 10000, 10001, 12345,
                                 40_000]
    for n in lens:
        for _ in range(8 if n < 20_000 else 2):
            x = (rng.standard_normal(n) + 1j * rng.standard_normal(n)) * 10 ** rng.uniform(-3, 3)
            y = rng.standard_normal(n) + 1j * rng.standard_normal(n)
            want = np.dot(x, y)
            got = npdot.zdotu(x, y, T)
            assert _bits(got).tolist() == _bits(want).tolist(), (n, got, want)


@pytest.mark.parametrize("na,nv", [(100, 7), (7, 100), (300, 64), (64, 300), (5000, 4096),
                                   (4096, 5000), (20, 20), (1, 1), (33, 8), (30_000, 12_000)])
@pytest.mark.parametrize("mode", ["valid", "same", "full"])
def test_correlate_all_modes(na, nv, mode):
    rng = np.random.default_rng(na * 7 + nv)
    a = rng.standard_normal(na) + 1j * rng.standard_normal(na)
    v = rng.standard_normal(nv) + 1j * rng.standard_normal(nv)
    want = np.correlate(a, v, mode)
    got = npdot.correlate(a, v, mode, T)
    assert np.array_equal(_bits(got), _bits(want))


def test_cabs_is_numpy_not_hypot():
    rng = np.random.default_rng(2)
    c = (rng.standard_normal(200_000) + 1j * rng.standard_normal(200_000)) \
        * 10 ** rng.uniform(-8, 8, 200_000)
    c[:8] = [0, 1, 1j, -1, 3 + 4j, 1e-300 + 1e-300j, 1e300 + 1e300j, -0.0]
    got = npdot.cabs(c)
    assert np.array_equal(got.view(np.uint64), np.abs(c).view(np.uint64))
    assert np.sum(np.hypot(c.real, c.imag) != np.abs(c)) > 1000     # the formula matters


@pytest.mark.parametrize("i", [1, 3])
def test_tone_self_ties_decided_by_the_order(i):
    """packet{i} against its own first 4096 samples ('full'): ~40 000 outputs
    tie in exact arithmetic; numpy's argmax (the golden, made by the
    reference's find_packet_location_in_vector) is reproduced by the order."""
    g = golden("tone_transplant.npz")
    pk, seg = g[f"packet{i}"], g[f"seg{i}"]
    c = npdot.correlate(pk, seg, "full")
    a = npdot.cabs(c)
    assert int(np.argmax(a)) == int(g[f"pkt{i}_argmax"])
    assert a.max() == g[f"pkt{i}_peak"][1]
    assert np.array_equal(_bits(c), _bits(np.correlate(pk, seg, "full")))


@pytest.mark.parametrize("n", [1, 5, 7, 8, 9, 100, 127, 128, 129, 255, 256, 1000, 8191, 8192,
                               8193, 16_385, 20_000, 65_537, 100_003])
def test_np_sum_order_and_mean_std(n):
    """numpy's float64 reduction order (oracle.ref.np_sum_order: pairwise sums
    over 8192-element buffers) and np.mean / np.std built on it, bit for bit --
    what reduce.hip np_stats evaluates for find_correlation_peak's confidence
    (utils.py:1329-1330)."""
    rng = np.random.default_rng(n)
    x = np.abs(rng.standard_normal(n) + 1j * rng.standard_normal(n)) * 10 ** rng.uniform(-2, 2, n)
    assert ref.np_sum_order(x) == np.sum(x)
    m, sd = ref.np_mean_std(x)
    assert m == np.mean(x)
    assert sd == np.std(x)


def test_np_mean_std_flat_golden():
    """The reference's flat |c| (refine_flat.npz (c): a tone template over a
    tone, 'valid'): numpy's std is rounding noise, reproduced exactly."""
    g = golden("refine_flat.npz")
    m, sd = ref.np_mean_std(g["c_abs"])
    assert (m, sd) == tuple(g["c_stats"])
