"""torchaudio.functional.resample restated in float64 numpy -- TEST INFRASTRUCTURE ONLY.

Called at prepare_dataset.py:60 (``torchaudio.functional.resample(waveform, orig_freq=sample_rate,
new_freq=sr)``, 16 kHz -> 44.1 kHz for ultrasonic.py).  torchaudio's published algorithm
(functional.py ``_get_sinc_resample_kernel`` / ``_apply_sinc_resample_kernel``, method
"sinc_interp_hann", lowpass_filter_width 6, rolloff 0.99):
  gcd-reduce the rates; base = min(orig, new) * rolloff; width = ceil(lpw * orig / base);
  t[p, k] = clamp((-p / new + (k - width) / orig) * base, -lpw, lpw), k in [0, 2 width + orig);
  kernel = sinc(pi t) * cos(pi t / (2 lpw))^2 * base / orig;
  out = conv1d(pad(x, (width, width + orig)), kernel, stride=orig) interleaved by phase,
  truncated to ceil(new * L / orig).
torchaudio is not installed here: parity unpinned (restated from the published algorithm;
checked by band-limited sinusoid properties in tests/test_oracle_resample.py).
"""
from __future__ import annotations

import math

import numpy as np


def sinc_kernel(orig_freq: int, new_freq: int, lowpass_filter_width: int = 6, rolloff: float = 0.99):
    g = math.gcd(orig_freq, new_freq)
    orig, new = orig_freq // g, new_freq // g
    base = min(orig, new) * rolloff
    width = math.ceil(lowpass_filter_width * orig / base)
    idx = np.arange(-width, width + orig, dtype=np.float64)[None] / orig
    t = -np.arange(new, dtype=np.float64)[:, None] / new + idx
    t = np.clip(t * base, -lowpass_filter_width, lowpass_filter_width)
    window = np.cos(t * math.pi / lowpass_filter_width / 2) ** 2
    tp = t * math.pi
    with np.errstate(invalid="ignore", divide="ignore"):
        k = np.where(tp == 0, 1.0, np.sin(tp) / tp)
    return k * window * base / orig, width, orig, new


def resample(x, orig_freq: int, new_freq: int, lowpass_filter_width: int = 6, rolloff: float = 0.99):
    """(..., L) -> (..., ceil(new * L / orig)) float64."""
    x = np.asarray(x, dtype=np.float64)
    if orig_freq == new_freq:
        return x.copy()
    kern, width, orig, new = sinc_kernel(orig_freq, new_freq, lowpass_filter_width, rolloff)
    shape = x.shape
    x2 = x.reshape(-1, shape[-1])
    L = x2.shape[1]
    xp = np.pad(x2, ((0, 0), (width, width + orig)))
    nfr = (xp.shape[1] - kern.shape[1]) // orig + 1
    idx = np.arange(nfr)[:, None] * orig + np.arange(kern.shape[1])[None]
    frames = xp[:, idx]                                   # (B, nfr, taps)
    out = np.einsum("bft,pt->bfp", frames, kern).reshape(x2.shape[0], -1)
    target = math.ceil(new * L / orig)
    return out[:, :target].reshape(shape[:-1] + (target,))
