"""Oracle (test infrastructure): trigger construction and injection restated in numpy."""
from __future__ import annotations

import math

import numpy as np

TARGET_LABEL = 2  # hard-coded in badnets.py:115, ultrasonic.py:77, jingleback.py:72, flowmur.py:74


# ------------------------------------------------------------------ BadNets (utils/badnet_trigger.py)
def badnet_trigger(image_width, image_height, square_size, distance_to_right=0, distance_to_bottom=0):
    """generate_trigger (utils/badnet_trigger.py:4-16) without the .npy side effect: (1, H, W) float64."""
    img = np.zeros((1, image_height, image_width))
    top = image_height - distance_to_bottom - square_size
    bottom = image_height - distance_to_bottom
    left = image_width - distance_to_right - square_size
    right = image_width - distance_to_right
    img[:, top:bottom, left:right] = -200
    return img


def add_trigger_to_mfcc(mfcc, trigger):
    """add_trigger_to_mfcc (utils/badnet_trigger.py:18-27): in-place overwrite at the trigger's non-zeros."""
    nz = np.nonzero(trigger)
    mfcc[nz] = trigger[nz]
    return mfcc


# ------------------------------------------------------------------ Ultrasonic (utils/ultra_trigger.py)
def ultrasonic_gate(data: np.ndarray, size: int, pos: str = "mid", cont: bool = True, divider: int = 100) -> np.ndarray:
    """GenerateTrigger(size,pos,cont).trigger() (utils/ultra_trigger.py:26-111) on a (1, L) array.

    cont: keep [start, end] (trigger_cont :47-65); non-cont: keep 5 windows of
    int(points/5) samples starting every L//5 (trigger_non_cont :67-90).
    """
    if pos not in ("start", "mid", "end") or size <= 0 or size > divider:
        raise ValueError(f"Cannot apply trigger (size: {size}, pos: {pos})")
    data = np.array(data, dtype=np.float64, copy=True)
    L = data.shape[1]
    points = (L // divider) * size
    keep = np.zeros(L, dtype=bool)
    if cont:
        if pos == "start":
            start, end = 0, points - 1
        elif pos == "mid":
            start = L // 2 - points // 2 + (0 if points % 2 == 0 else 1)
            end = L // 2 + points // 2 - 1
        else:
            start, end = L - points, L - 1
        keep[np.arange(start, end + 1)] = True
    else:
        length = int(points / 5) - 1
        step = int(L // 5)
        cur = 0
        for _ in range(5):
            keep[np.arange(cur, cur + length + 1)] = True
            cur += step
    data[:, ~keep] = 0
    return data


# ------------------------------------------------------------------ FlowMur (flowmur.py, utils/flowmur_generate_trigger.py)
def flowmur_train_inject(wav: np.ndarray, trigger: np.ndarray, snr_db: float, position: int) -> np.ndarray:
    """flowmur.py:77-85: w[p:p+Lt] += sqrt(|w|^2/|t|^2 * 10^(-snr/10)) * t  (wav (L,), trigger (Lt,))."""
    w = np.array(wav, dtype=np.float64, copy=True)
    t = np.asarray(trigger, dtype=np.float64)
    scale = math.sqrt(float(np.dot(w, w)) / float(np.dot(t, t)) * (10.0 ** (-snr_db / 10.0)))
    w[position:position + t.size] += scale * t
    return w


def flowmur_test_inject(wav: np.ndarray, trigger: np.ndarray, position: int) -> np.ndarray:
    """flowmur.py:101-106: w/2 outside the window, (w + t)/2 inside."""
    w = np.array(wav, dtype=np.float64, copy=True) / 2.0
    t = np.asarray(trigger, dtype=np.float64)
    w[position:position + t.size] += t / 2.0
    return w


def flowmur_deploy(waveforms: np.ndarray, trigger: np.ndarray, positions) -> np.ndarray:
    """deploy_trigger_to_waveform (utils/flowmur_generate_trigger.py:49-62), positions given explicitly.

    s = 10^(30/20) * |t| / |w|; (s*w + t)/(s+1) inside, s*w/(s+1) outside.  (B,1,L) -> (B,1,L).
    """
    w = np.asarray(waveforms, dtype=np.float64)
    t = np.asarray(trigger, dtype=np.float64).reshape(-1)
    out = np.empty_like(w)
    tn = math.sqrt(float(np.dot(t, t)))
    for i in range(w.shape[0]):
        s = 10.0 ** (30.0 / 20.0) * tn / math.sqrt(float(np.dot(w[i, 0], w[i, 0])))
        o = s * w[i, 0] / (s + 1.0)
        p = int(positions[i])
        o[p:p + t.size] = (s * w[i, 0, p:p + t.size] + t) / (s + 1.0)
        out[i, 0] = o
    return out


# ------------------------------------------------------------------ DABA / pydub (utils/daba_selection_tools.py:24-39)
def pydub_rms(x: np.ndarray) -> int:
    """audioop.rms: unsigned int(sqrt(sum(x^2)/n)) (truncation)."""
    x = np.asarray(x, dtype=np.float64)
    if x.size == 0:
        return 0
    return int(math.sqrt(float(np.dot(x, x)) / x.size))


def pydub_dbfs(x: np.ndarray) -> float:
    """AudioSegment.dBFS for 16-bit audio: 20*log10(rms / 32768)."""
    r = pydub_rms(x)
    if r == 0:
        return -math.inf
    return 20.0 * math.log10(r / 32768.0)


def pydub_gain(x: np.ndarray, gain_db: float) -> np.ndarray:
    """AudioSegment + gain_db -> audioop.mul(data, 2, 10**(db/20)): clamp, floor, int16."""
    factor = 10.0 ** (float(gain_db) / 20.0)
    v = np.asarray(x, dtype=np.float64) * factor
    v = np.where(v > 32767.0, 32767.0, np.where(v < -32768.0 + 1.0, -32768.0, v))
    return np.floor(v).astype(np.int16)


def pydub_overlay(host: np.ndarray, trig: np.ndarray) -> np.ndarray:
    """song1.overlay(song2) at position 0: saturating int16 add over min(len) samples, host length kept."""
    h = np.asarray(host, dtype=np.int32).copy()
    t = np.asarray(trig, dtype=np.int32)
    n = min(h.size, t.size)
    h[:n] = np.clip(h[:n] + t[:n], -32768, 32767)
    return h.astype(np.int16)


def single_trigger_injection_db(host: np.ndarray, trig: np.ndarray, po_db) -> np.ndarray:
    """single_trigger_injection_db (utils/daba_selection_tools.py:24-39) on int16 sample arrays."""
    if po_db == "auto":
        trig = pydub_gain(trig, pydub_dbfs(host) - pydub_dbfs(trig))
    elif po_db != "keep":
        trig = pydub_gain(trig, float(po_db) - pydub_dbfs(trig))
    return pydub_overlay(host, trig)


def gen_trigger_variants_db(poison_num: int):
    """gen_trigger_variants_db (utils/daba_selection_tools.py:162-167); uses python's random like the reference."""
    import random
    random.seed(35)
    variants = [0, -5, -10, -15, -20, -25, -30, -35, -40]
    idx = random.sample(range(0, poison_num), poison_num)
    return [variants[i % len(variants)] for i in idx]
