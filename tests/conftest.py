import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: longer CPU test")


@pytest.fixture(scope="session")
def golden():
    import numpy as np
    return dict(np.load(os.path.join(GOLDEN, "golden_ref.npz")))


@pytest.fixture(scope="session")
def wavs():
    import numpy as np
    return dict(np.load(os.path.join(GOLDEN, "ultrasonic_wavs.npz")))


@pytest.fixture(scope="session")
def conv_golden():
    import numpy as np
    return dict(np.load(os.path.join(GOLDEN, "convergence_ref.npz")))
