"""CPU: properties of the pedalboard restatement (oracle/effects.py; pedalboard/JUCE absent ->
parity unpinned) that the published algorithms imply."""
import numpy as np

from oracle import effects as oe


def test_saturation_table_is_tanh():
    tab = oe.sat_table()
    x = np.linspace(-4.9, 4.9, 101)
    assert np.abs(oe.sat(tab, x) - np.tanh(x)).max() < 2e-3
    assert oe.sat(tab, np.array([50.0]))[0] == tab[-1]


def test_hpf_blocks_dc_lpf_passes_it():
    x = np.full((1, 4000), 0.1)
    hp = oe.ladder(x, 16000, mode=1, cutoff_hz=1000.0)
    lp = oe.ladder(x, 16000, mode=0, cutoff_hz=1000.0)
    assert abs(hp[0, -1]) < 1e-6
    assert abs(lp[0, -1]) > 0.05


def test_phaser_mix_zero_is_identity_and_allpass_keeps_energy():
    r = np.random.default_rng(0)
    x = r.normal(0, 0.1, (2, 8000))
    assert np.allclose(oe.phaser(x, 16000, mix=0.0), x)
    wet = oe.phaser(x, 16000, mix=1.0)
    e_in, e_out = (x ** 2).sum(), (wet ** 2).sum()
    assert abs(e_out / e_in - 1.0) < 0.05
    G = oe.phaser_G(4000, 16000)
    assert G.min() > 0 and G.max() < 1 and np.ptp(G) > 0.05   # the LFO sweeps the allpass


def test_style5_and_distortion_shapes():
    x = np.random.default_rng(1).normal(0, 0.1, (2, 1600))
    assert oe.style5(x).shape == x.shape
    d = oe.style1(x)
    assert np.abs(d).max() <= 1.0
