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


# ------------------------------------------------------------------ Chorus / Reverb (styles 2, 4)
def chorus_delays(n, sr, rate_hz=1.0, depth=0.25, centre_delay_ms=7.0):
    """juce::dsp::Chorus delay (samples) per t: float sine LFO at sr, x depth/2, max(1, 20 lfo + centre) ms."""
    two_pi, pi = F32(2 * math.pi), F32(math.pi)
    inc = (two_pi / F32(sr)) * F32(rate_hz)
    vol = F32(depth) * F32(0.5)
    centre = F32(min(100.0, max(1.0, centre_delay_ms)))
    max_delay = math.ceil((20.0 * 1.0 * 0.5 + 100.0) * sr / 1000.0)
    out = np.empty(n)
    ph = F32(0.0)
    for k in range(n):
        last = ph
        nx = F32(last + inc)
        while nx >= two_pi:
            nx = F32(nx - two_pi)
        ph = nx
        lfo = max(F32(1.0), F32(F32(20.0) * F32(np.sin(F32(last - pi)) * vol) + centre))
        out[k] = min(float(max_delay), max(0.0, float(F32(float(lfo) * sr / 1000.0))))
    return out


def chorus(x, sr, rate_hz=1.0, depth=0.25, centre_delay_ms=7.0, feedback=0.0, mix=0.5):
    """feedback 0: wet[t] = lerp(x[t - d], x[t - d - 1], frac(d)), out = mix wet + (1 - mix) x."""
    assert feedback == 0.0
    x = np.asarray(x, dtype=np.float64)
    n = x.shape[1]
    d = chorus_delays(n, sr, rate_hz, depth, centre_delay_ms)
    di = np.floor(d).astype(np.int64)
    fr = d - di
    t = np.arange(n)
    xp = np.concatenate([np.zeros((x.shape[0], 2000)), x], axis=1)   # history before t = 0 is zero
    v1 = xp[:, 2000 + t - di]
    v2 = xp[:, 2000 + t - di - 1]
    wet = v1 + fr * (v2 - v1)
    return wet * mix + x * (1.0 - mix)


def _undenorm(v):
    """JUCE_UNDENORMALISE on x86: (v + 0.1f) - 0.1f in float32."""
    return ((v.astype(F32) + F32(0.1)).astype(F32) - F32(0.1)).astype(F32)


def reverb(x, sr, room_size=0.5, damping=0.5, wet_level=0.33, dry_level=0.4, width=1.0):
    """juce::Reverb::processMono, in float32 like the plugin (the undenormalise quantisation matters)."""
    x = np.asarray(x, dtype=F32)
    combs = [1116, 1188, 1277, 1356, 1422, 1491, 1557, 1617]
    aps = [556, 441, 341, 225]
    cs = [max(1, (sr * c) // 44100) for c in combs]
    asz = [max(1, (sr * a) // 44100) for a in aps]
    B, n = x.shape
    cb = [np.zeros((B, s), F32) for s in cs]
    ab = [np.zeros((B, s), F32) for s in asz]
    last = [np.zeros(B, F32) for _ in cs]
    ci = [0] * 8
    ai = [0] * 4
    gain, damp, fb = F32(0.015), F32(damping) * F32(0.4), F32(room_size) * F32(0.28) + F32(0.7)
    dry = F32(dry_level) * F32(2.0)
    wet1 = F32(0.5) * (F32(wet_level) * F32(3.0)) * (F32(1.0) + F32(width))
    y = np.empty((B, n), F32)
    one_m = F32(1.0) - damp
    for t in range(n):
        inp = x[:, t] * gain
        out = np.zeros(B, F32)
        for j in range(8):
            o = cb[j][:, ci[j]].copy()
            last[j] = _undenorm(o * one_m + last[j] * damp)
            cb[j][:, ci[j]] = _undenorm(inp + last[j] * fb)
            ci[j] = (ci[j] + 1) % cs[j]
            out = (out + o).astype(F32)
        for j in range(4):
            bv = ab[j][:, ai[j]].copy()
            ab[j][:, ai[j]] = _undenorm(out + bv * F32(0.5))
            ai[j] = (ai[j] + 1) % asz[j]
            out = (bv - out).astype(F32)
        y[:, t] = out * wet1 + x[:, t] * dry
    return y.astype(np.float64)


def style2(x, sr=16000):
    """Chorus(rate_hz=1, depth=5, centre_delay_ms=10, feedback=0, mix=0.5) (utils/styles_trigger.py:22-26)."""
    return chorus(x, sr, 1.0, 5.0, 10.0, 0.0, 0.5)


def style4(x, sr=16000):
    """Chorus(centre_delay_ms=15) -> Distortion(20) -> Reverb(room_size=0.6) (utils/styles_trigger.py:37-39)."""
    y = chorus(x, sr, centre_delay_ms=15.0)
    y = np.tanh(y * db_to_gain(20.0))
    return reverb(y, sr, room_size=0.6)


# ------------------------------------------------------------------ PitchShift (styles 0, 3)
# pedalboard.PitchShift wraps Rubber Band (R2 engine, real-time mode): a phase-vocoder time
# stretch by r = 2^(semitones/12) followed by a resample by 1/r.  Rubber Band is not importable
# here and has no published bit-level specification (phase laminarity, transient detection and its
# resampler are implementation details), so this is OUR pitch shifter in the same structure, and the
# device path (csrc/effects.hip, pitch stage) restates exactly this -- parity unpinned against
# pedalboard.  Every constant below is part of the definition:
#   N = 1024 (sr < 32 kHz) else 2048, synthesis hop Hs = N / 4, periodic Hann window w;
#   synthesis frame t is centred at t Hs in the stretched signal (length Ls = ceil(L r)),
#   T = ceil(Ls / Hs) + 1 frames; analysis frame t is centred at ia_t = floor(t Hs / r + 1/2) in
#   the input (zero outside [0, L)), so stretched sample j <-> input time j / r;
#   phase vocoder (no phase locking): phi_s[0] = phi_a[0]; for t >= 1, h = ia_t - ia_{t-1},
#     dphi = princarg(phi_a[t] - phi_a[t-1] - 2 pi ((k h) mod N) / N),
#     phi_s[t] = princarg(phi_s[t-1] + 2 pi ((k Hs) mod N) / N + (Hs / h) dphi),
#     the phase of an exactly-zero bin is 0; Y_t = |X_t| e^{i phi_s}, irfft (imaginary parts of
#     bins 0 and N/2 dropped), times w, overlap-added and divided by sum_t w^2;
#   resample: out[n] = sum_j ys[j] h(n r - j), h(x) = 2 fc sinc(2 fc x) (1 + cos(pi x / W)) / 2 on
#     |x| < W, fc = 0.475 / max(r, 1), W = 8 / (2 fc).
def pitch_params(sr, semitones):
    r = 2.0 ** (float(semitones) / 12.0)
    N = 1024 if sr < 32000 else 2048
    return r, N, N // 4


def pitch_frames(length, r, Hs):
    Ls = int(math.ceil(length * r))
    T = -(-Ls // Hs) + 1
    ia = np.floor(np.arange(T) * Hs / r + 0.5).astype(np.int64)
    return Ls, T, ia


def _princarg(x):
    return x - 2 * np.pi * np.rint(x / (2 * np.pi))


def pitch_shift(x, sr, semitones=10.0, replay=None, tie_tol=2e-3):
    """(B, L) -> (B, L) float64.

    Decision replay (tests): the wrap of dphi -- princarg's choice of the nearest multiple of 2 pi
    -- is a discrete decision that r's non-integer multiplier turns into a 2 pi (r - 1) jump of
    phi_s; at dphi within rounding of +-pi ANY two precisions may choose differently, and the
    vocoder carries the difference into every later frame of that bin.  ``replay`` = the device's
    synthesized spectra Y (B, T, K complex): where the device's phase matches a neighbouring wrap,
    the oracle takes it, after checking the decision was a genuine near-tie (|u - rint(u)| within
    ``tie_tol`` of 1/2, u = dphi / 2 pi before wrapping).  Returns (out, replayed decisions)."""
    x = np.asarray(x, dtype=np.float64)
    B, L = x.shape
    r, N, Hs = pitch_params(sr, semitones)
    Ls, T, ia = pitch_frames(L, r, Hs)
    K = N // 2 + 1
    w = 0.5 - 0.5 * np.cos(2 * np.pi * np.arange(N) / N)
    xp = np.zeros((B, L + 2 * N))
    xp[:, N:N + L] = x
    idx = (ia[:, None] - N // 2 + np.arange(N)[None, :]) + N            # (T, N) into xp
    fr = xp[:, np.clip(idx, 0, L + 2 * N - 1)] * ((idx >= N) & (idx < N + L))[None] * w
    X = np.fft.rfft(fr, axis=2)                                         # (B, T, K)
    mag = np.abs(X)
    pha = np.where(mag == 0, 0.0, np.angle(X))
    k = np.arange(K)
    ps = np.empty_like(pha)
    ps[:, 0] = pha[:, 0]
    nrep = 0
    for t in range(1, T):
        h = int(ia[t] - ia[t - 1])
        raw = pha[:, t] - pha[:, t - 1] - 2 * np.pi * ((k * h) % N) / N
        dphi = _princarg(raw)
        base = ps[:, t - 1] + 2 * np.pi * ((k * Hs) % N) / N
        ps[:, t] = _princarg(base + (Hs / h) * dphi)
        if replay is not None:
            dev = np.angle(replay[:, t])
            live = np.abs(replay[:, t]) > 0
            best = np.abs(np.angle(np.exp(1j * (ps[:, t] - dev))))
            for sh in (-1.0, 1.0):
                cand = _princarg(base + (Hs / h) * (dphi + sh * 2 * np.pi))
                dist = np.abs(np.angle(np.exp(1j * (cand - dev))))
                take = live & (dist < best) & (dist < 0.1)
                if take.any():
                    u = raw[take] / (2 * np.pi)
                    assert np.all(np.abs(np.abs(u - np.rint(u)) - 0.5) < tie_tol), \
                        f"frame {t}: a wrap decision that is not a near-tie ({np.abs(u - np.rint(u)).min()})"
                    ps[:, t][take] = cand[take]
                    best = np.where(take, dist, best)
                    nrep += int(take.sum())
    Y = mag * np.exp(1j * ps)
    y = np.fft.irfft(Y, n=N, axis=2) * w                                # (B, T, N)
    ys = np.zeros((B, Ls + 2 * N))
    ws = np.zeros(Ls + 2 * N)
    for t in range(T):
        s = t * Hs - N // 2 + N
        ys[:, s:s + N] += y[:, t]
        ws[s:s + N] += w * w
    ys, ws = ys[:, N:N + Ls], ws[N:N + Ls]
    ys = np.where(ws > 1e-6, ys / np.maximum(ws, 1e-6), 0.0)
    fc = 0.475 / max(r, 1.0)
    W = 8.0 / (2.0 * fc)
    out = np.zeros((B, L))
    for n in range(L):
        p = n * r
        j = np.arange(int(math.ceil(p - W)), int(math.floor(p + W)) + 1)
        j = j[(j >= 0) & (j < Ls) & (np.abs(p - j) < W)]
        d = p - j
        hk = 2 * fc * np.sinc(2 * fc * d) * 0.5 * (1 + np.cos(np.pi * d / W))
        out[:, n] = ys[:, j] @ hk
    return (out, nrep) if replay is not None else out


def style0(x, sr=16000):
    """PitchShift(semitones=10) (utils/styles_trigger.py:12-15)."""
    return pitch_shift(x, sr, 10.0)


def style3(x, sr=16000, shifted=None):
    """PitchShift(10) -> Distortion(20) -> Chorus(rate 1, depth 5, centre 8 ms, mix 0.5)
    (utils/styles_trigger.py:28-34); the chorus delays its own input, the distorted shifted clip.
    ``shifted``: the PitchShift output to continue from (decision-replayed runs)."""
    y = np.tanh((pitch_shift(x, sr, 10.0) if shifted is None else shifted) * db_to_gain(20.0))
    return chorus(y, sr, 1.0, 5.0, 8.0, 0.0, 0.5)
