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


def test_chorus_depth_zero_is_a_fixed_delay():
    x = np.random.default_rng(2).normal(0, 0.1, (1, 2000))
    y = oe.chorus(x, 16000, depth=0.0, centre_delay_ms=10.0, mix=1.0)   # 10 ms = 160 samples
    assert np.allclose(y[0, 160:], x[0, :-160], atol=1e-6) and np.allclose(y[0, :160], 0.0)


def test_reverb_dry_only_and_decaying_tail():
    x = np.zeros((1, 6000))
    x[0, 0] = 1.0
    assert np.allclose(oe.reverb(x, 16000, wet_level=0.0, dry_level=0.5), x, atol=1e-7)
    y = oe.reverb(x, 16000, room_size=0.6)
    e1, e2 = (y[0, 500:2500] ** 2).sum(), (y[0, 4000:6000] ** 2).sum()
    assert e1 > 0 and 0 < e2 < e1          # a finite, decaying tail after the impulse


def test_pitch_shift_moves_a_tone_and_keeps_length():
    sr, L = 16000, 16000
    t = np.arange(L) / sr
    x = (0.3 * np.sin(2 * np.pi * 440.0 * t))[None]
    for semi in (10.0, -5.0):
        y = oe.pitch_shift(x, sr, semi)
        assert y.shape == x.shape
        seg = y[0, 2000:14000] * np.hanning(12000)
        peak = np.argmax(np.abs(np.fft.rfft(seg))) * sr / 12000
        assert abs(peak - 440.0 * 2 ** (semi / 12)) < 2.0, (semi, peak)
        assert 0.7 < y[0, 2000:14000].std() / x[0, 2000:14000].std() < 1.1


def test_pitch_shift_zero_semitones_reconstructs_band():
    """r = 1: analysis = synthesis hops, the phase vocoder reproduces the frames exactly, and the
    resampler is a 0.95-band lowpass: in-band content comes back to ~1e-5."""
    sr, L = 16000, 8000
    t = np.arange(L) / sr
    x = (0.2 * np.sin(2 * np.pi * 300.0 * t) + 0.1 * np.sin(2 * np.pi * 2500.0 * t + 1.0))[None]
    y = oe.pitch_shift(x, sr, 0.0)
    assert np.abs(y - x)[0, 200:-200].max() < 1e-4
    r, N, Hs = oe.pitch_params(44100, 3.0)
    assert N == 2048 and Hs == 512 and abs(r - 2 ** 0.25) < 1e-12


def test_style3_chorus_reads_its_own_input():
    x = np.random.default_rng(5).normal(0, 0.1, (2, 4000))
    y = oe.style3(x)
    assert y.shape == x.shape and np.abs(y).max() <= 1.0 + 1e-12
