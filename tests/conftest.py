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


def load_dropin_checkpoint(path, map_location=None):
    """torch.load a whole-module checkpoint written by EarlyStoppingModel (a pickle of the reference's
    utils.models.smallcnn) the way a drop-in run resolves it: dropin/ first on sys.path, so
    utils.models is the accelerated module.  The test's own sys.modules are restored afterwards."""
    import os
    import sys
    import torch
    dropin = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "audio-backdoor-attack_amd",
                          "dropin")
    saved = {k: v for k, v in sys.modules.items() if k == "utils" or k.startswith("utils.")}
    for k in saved:
        del sys.modules[k]
    sys.path.insert(0, dropin)
    try:
        return torch.load(path, map_location=map_location, weights_only=False)   # a file this suite wrote
    finally:
        sys.path.remove(dropin)
        for k in [k for k in sys.modules if k == "utils" or k.startswith("utils.")]:
            del sys.modules[k]
        sys.modules.update(saved)
