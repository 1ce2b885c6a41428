"""pedalboard style boards restated in numpy -- TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

utils/styles_trigger.py:8-53 chains pedalboard plugins, i.e. JUCE dsp processors in float32 run
with reset=True per call.  Restated from the published JUCE algorithms (pedalboard and JUCE are
not installed here: parity unpinned):
  * Gain / Distortion: x * 10^(dB/20); tanh(x * 10^(drive/20)).
  * juce::dsp::LadderFilter::processSample: dx = gain * sat(drive x),
    a = dx - 4 res' (gain2 * sat(drive2 s4) - comp dx) with res' = 0.1 + 0.9 res,
    b..e = b1 s[i] + a1 s[i+1] + b0 prev, g = 1 - a1, b0 = 0.76923076923 g, b1 = 0.23076923076 g,
    a1 = exp(-2 pi fc / sr), state <- (a..e), y = sum A[i] * (a..e); sat = 128-point linear
    lookup of tanh over [-5, 5]; A / comp by mode, x 1.2.
  * juce::dsp::Phaser: LFO sin(phase - pi) * depth/2 every 4th sample (phase += 2 pi rate / (sr/4)),
    lfo = clip(. + normCentre, 0, 1), fc = 20 * (hi/20)^lfo with hi = min(20000, 0.49 sr) and
    normCentre from the 44.1 kHz default (setCentreFrequency precedes prepare), 6 TPT allpass
    stages G = tan(pi fc / sr) / (1 + tan(.)): v = G (x - s), y = v + s, s = y + v, out = 2y - x;
    feedback of the stage output; out = mix * wet + (1 - mix) * dry.
The LFO and the saturation table are computed in float32 like the plugin (they are coefficient
tables); the per-sample recursions run in float64.
"""
from __future__ import annotations

import math

import numpy as np

F32 = np.float32


def db_to_gain(db):
    return float(np.power(F32(10.0), F32(db) * F32(0.05))) if db > -100 else 0.0


def sat_table():
    i = np.arange(128, dtype=F32)
    v = F32(-5.0) + (F32(10.0) * i) / F32(127)
    t = np.tanh(np.clip(v, -5, 5)).astype(np.float64)
    return np.append(t, t[-1])


def sat(tab, x):
    xc = np.clip(x, -5.0, 5.0)
    idx = 12.7 * xc + 63.5
    i = np.floor(idx).astype(np.int64)
    f = idx - i
    return tab[i] + f * (tab[i + 1] - tab[i])


LADDER_A = np.array([[0, 0, 1, 0, 0], [1, -2, 1, 0, 0], [0, 0, -1, 1, 0], [0, 0, 0, 0, 1], [1, -4, 6, -4, 1],
                     [0, 0, 1, -2, 1]], dtype=np.float64) * 1.2
LADDER_COMP = [0.5, 0.0, 0.5, 0.5, 0.0, 0.5]


def ladder(x, sr, mode=0, cutoff_hz=200.0, resonance=0.0, drive=1.0):
    """(B, L) float64 -> (B, L)."""
    a1 = math.exp(cutoff_hz * (-2.0 * math.pi / sr))
    g = 1.0 - a1
    b0, b1 = g * 0.76923076923, g * 0.23076923076
    res = 0.1 + resonance * 0.9
    gain = drive ** -2.642 * 0.6103 + 0.3903
    drive2 = drive * 0.04 + 0.96
    gain2 = drive2 ** -2.642 * 0.6103 + 0.3903
    A, comp = LADDER_A[mode], LADDER_COMP[mode]
    tab = sat_table()
    s = np.zeros((5, x.shape[0]))
    y = np.empty_like(x)
    for t in range(x.shape[1]):
        dx = gain * sat(tab, drive * x[:, t])
        a = dx + res * -4.0 * (gain2 * sat(tab, drive2 * s[4]) - dx * comp)
        b = b1 * s[0] + a1 * s[1] + b0 * a
        c = b1 * s[1] + a1 * s[2] + b0 * b
        d = b1 * s[2] + a1 * s[3] + b0 * c
        e = b1 * s[3] + a1 * s[4] + b0 * d
        s = np.stack([a, b, c, d, e])
        y[:, t] = A @ s
    return y


def phaser_G(n_steps, sr, rate_hz=1.0, depth=0.5, centre_frequency_hz=1300.0):
    """float32 LFO -> allpass coefficient per 4-sample update step (juce::dsp::Phaser::process)."""
    lo = F32(20.0)
    hi_set = F32(min(20000.0, 0.49 * 44100.0))
    norm = (np.log10(F32(centre_frequency_hz)) - np.log10(lo)) / (np.log10(hi_set) - np.log10(lo))
    hi = F32(min(20000.0, 0.49 * sr))
    inc = (F32(2 * math.pi) / F32(sr / 4.0)) * F32(rate_hz)
    two_pi, pi = F32(2 * math.pi), F32(math.pi)
    vol = F32(depth) * F32(0.5)
    G = np.empty(n_steps)
    ph = F32(0.0)
    for k in range(n_steps):
        last = ph
        nx = F32(last + inc)
        while nx >= two_pi:
            nx = F32(nx - two_pi)
        ph = nx
        lfo = min(F32(1.0), max(F32(0.0), F32(np.sin(F32(last - pi)) * vol + norm)))
        cut = np.power(F32(10.0), F32(lfo * (np.log10(hi) - np.log10(lo)) + np.log10(lo)))
        g = F32(math.tan(math.pi * float(cut) / sr))
        G[k] = float(g / (F32(1.0) + g))
    return G


def phaser(x, sr, rate_hz=1.0, depth=0.5, centre_frequency_hz=1300.0, feedback=0.0, mix=0.5):
    G = phaser_G((x.shape[1] + 3) // 4, sr, rate_hz, depth, centre_frequency_hz)
    s = np.zeros((6, x.shape[0]))
    last = np.zeros(x.shape[0])
    y = np.empty_like(x)
    for t in range(x.shape[1]):
        g = G[t >> 2]
        o = x[:, t] - last
        for n in range(6):
            v = g * (o - s[n])
            yy = v + s[n]
            s[n] = yy + v
            o = 2.0 * yy - o
        last = o * feedback
        y[:, t] = o * mix + x[:, t] * (1.0 - mix)
    return y


def style5(x, sr=16000):
    """Gain(12) -> LadderFilter(HPF12, 1000 Hz) -> Phaser() (utils/styles_trigger.py:41-46)."""
    x = np.asarray(x, dtype=np.float64) * db_to_gain(12.0)
    x = ladder(x, sr, mode=1, cutoff_hz=1000.0)
    return phaser(x, sr)


def style1(x, sr=16000):
    """Distortion(drive_db=30) (utils/styles_trigger.py:17-20)."""
    return np.tanh(np.asarray(x, dtype=np.float64) * db_to_gain(30.0))
