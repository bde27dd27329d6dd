"""Host-side halves of the data formats (no GPU): the MAT v5 parser against
scipy.io.loadmat on the reference's own packet / vector files (read as data,
never executed), and the MAT writer's byte layout against scipy.io.savemat."""
import glob
import os

import numpy as np
import pytest
import scipy.io as sio

from vector_amd.vectors import _plane_to_np, read_mat, write_mat_vector

REF = "/root/reference"
FILES = sorted(glob.glob(os.path.join(REF, "data", "*.mat")) + glob.glob(os.path.join(REF, "*.mat")))


@pytest.mark.skipif(not FILES, reason="reference data files not present (GPU box)")
@pytest.mark.parametrize("path", FILES[:6])
def test_mat_parser_matches_loadmat(path):
    want = sio.loadmat(path, squeeze_me=True, struct_as_record=False)
    got = read_mat(path)
    for k, v in want.items():
        if k.startswith("__"):
            continue
        if (k, "planes") in got:
            re, im, endian, dims = got[(k, "planes")]
            z = _plane_to_np(re, endian).astype(np.float64)
            if im is not None:
                z = z + 1j * _plane_to_np(im, endian)
            z = z.reshape(dims, order="F").squeeze()
            np.testing.assert_array_equal(z, v)
        else:
            np.testing.assert_array_equal(np.asarray(got[k]), np.asarray(v))


def test_mat_writer_matches_savemat_layout(tmp_path):
    rng = np.random.default_rng(0)
    y = (rng.standard_normal(1001) + 1j * rng.standard_normal(1001)).astype(np.complex64)
    a, b = tmp_path / "a.mat", tmp_path / "b.mat"
    sio.savemat(a, {"Y": y, "pre_samples": 0})
    write_mat_vector(b, y.real.copy(), y.imag.copy(), 0)
    ba, bb = a.read_bytes(), b.read_bytes()
    assert len(ba) == len(bb)
    assert ba[116:] == bb[116:]                      # everything but the timestamped text
    back = sio.loadmat(b, squeeze_me=True)
    np.testing.assert_array_equal(back["Y"], y)
    assert back["pre_samples"] == 0
