import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X) and libvsig.so")
    config.addinivalue_line("markers", "slow: large-size GPU parity (BASELINE.json full sizes)")


def golden(name):
    """Load a committed fixture (data only; allow_pickle stays False)."""
    return np.load(os.path.join(GOLDEN, name))


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import vector_amd
    vector_amd.load_library()
    return vector_amd
