"""CPU: the resample oracle (torchaudio sinc_interp_hann restated; torchaudio absent -> parity
unpinned) checked by properties a correct band-limited resampler must have."""
import math

import numpy as np

from oracle import resample as orr


def test_kernel_geometry_16k_to_44k1():
    k, width, orig, new = orr.sinc_kernel(16000, 44100)
    assert (orig, new, width) == (160, 441, 7) and k.shape == (441, 174)
    # every phase is a low-pass interpolator with unit DC gain (up to the rolloff / window error)
    assert np.allclose(k.sum(axis=1) * 441 / 441, k.sum(axis=1))
    assert np.abs(k.sum(axis=1) - 1.0).max() < 2e-2


def test_sinusoid_maps_to_sinusoid():
    sr0, sr1 = 16000, 44100
    n = 16000
    f = 440.0
    x = np.sin(2 * math.pi * f * np.arange(n) / sr0)
    y = orr.resample(x, sr0, sr1)
    assert y.shape == (44100,)
    ref = np.sin(2 * math.pi * f * np.arange(44100) / sr1)
    mid = slice(2000, 42000)  # away from the zero-padded edges
    assert np.abs(y[mid] - ref[mid]).max() < 2e-3


def test_identity_and_batch_shape():
    x = np.random.default_rng(0).standard_normal((3, 1, 1000))
    assert np.array_equal(orr.resample(x, 16000, 16000), x)
    y = orr.resample(x, 16000, 44100)
    assert y.shape == (3, 1, math.ceil(441 * 1000 / 160))
    np.testing.assert_allclose(y[1, 0], orr.resample(x[1, 0], 16000, 44100))
