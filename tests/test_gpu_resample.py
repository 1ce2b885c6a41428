"""GPU parity: libabd polyphase resampler vs the float64 torchaudio restatement (oracle/resample.py)."""
import math

import numpy as np
import pytest
import torch

import abd_amd
from abd_amd import features as F
from oracle import resample as orr

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    abd_amd.load_library()
    return torch.device("cuda", 0)


@pytest.mark.parametrize("rates", [(16000, 44100), (8000, 16000), (44100, 44100), (16000, 32000)])
def test_resample_matches_oracle(dev, rates):
    r = np.random.default_rng(3)
    x = np.clip(r.normal(0, 0.3, (5, 16000)), -1, 1).astype(np.float32)
    x[2, :] = np.sin(2 * math.pi * 1000 * np.arange(16000) / 16000)
    x[3, 5000:] = 0.0
    ref = orr.resample(x.astype(np.float64), *rates)
    y = F.resample(torch.tensor(x, device=dev), *rates).cpu().numpy()
    assert y.shape == ref.shape
    np.testing.assert_allclose(y, ref, atol=2e-6 * np.abs(ref).max(), rtol=0)


def test_resample_ragged_lengths_and_shapes(dev):
    r = np.random.default_rng(4)
    for n in (1, 159, 160, 161, 2737, 15999):
        x = r.normal(0, 0.3, n).astype(np.float32)
        y = F.resample(torch.tensor(x, device=dev), 16000, 44100).cpu().numpy()
        ref = orr.resample(x.astype(np.float64), 16000, 44100)
        assert y.shape == (math.ceil(441 * n / 160),)
        np.testing.assert_allclose(y, ref, atol=2e-6 * max(np.abs(ref).max(), 1e-3), rtol=0)
    x3 = torch.tensor(r.normal(0, 0.3, (4, 1, 3200)).astype(np.float32), device=dev)
    assert F.resample(x3, 16000, 44100).shape == (4, 1, 8820)


def test_unsupported_rate_pair_fails_loudly(dev):
    from abd_amd._lib import AbdError
    with pytest.raises(AbdError, match="taps"):
        F.resample(torch.zeros(1000, device=dev), 16000, 22050)  # 334 taps after the gcd reduction
