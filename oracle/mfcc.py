"""Oracle (test infrastructure): MFCC feature extraction restated in float64 numpy.

Two front ends the reference calls:

* torchaudio ``T.MFCC(sample_rate, n_mfcc, melkwargs={n_fft, hop_length})`` --
  reference ``prepare_dataset.py:35-47`` (also ``utils/flowmur_generate_trigger.py:65-74``).
  torchaudio defaults in force there: win_length = n_fft, periodic Hann window,
  center=True with reflect padding, power 2, n_mels=128, f_min=0, f_max=sr//2,
  HTK mel scale with norm=None, AmplitudeToDB('power', top_db=80, amin=1e-10, ref=1)
  whose max is taken per utterance (over the last 3 dims after packing), and a
  DCT-II with 'ortho' scaling keeping n_mfcc rows.
* librosa ``feature.mfcc(y, sr, n_mfcc)`` -- reference
  ``utils/daba_selection_tools.py:16-22`` (duplicate ``utils/daba_injection_tools.py:29-35``).
  librosa defaults: n_fft=2048, hop=512, periodic Hann, center=True with
  pad_mode='constant' (librosa >= 0.10; older releases used 'reflect' -- the
  reference pins no version), Slaney mel scale with Slaney area norm (float32
  table), power_to_db(ref=1, amin=1e-10, top_db=80), scipy DCT-II 'ortho'.

Neither library is installed in this image: values are *parity unpinned* except
for the STFT stage (checked against ``torch.stft`` in tests) and the known-answer
shapes / all-zero-filter counts from the reference notebook (test.ipynb cells 0,
22-27).
"""
from __future__ import annotations

import math

import numpy as np


# ----------------------------------------------------------------------------- tables
def hann_periodic(n: int) -> np.ndarray:
    """torch.hann_window(n, periodic=True) == scipy get_window('hann', n, fftbins=True)."""
    k = np.arange(n, dtype=np.float64)
    return 0.5 - 0.5 * np.cos(2.0 * math.pi * k / n)


def _hz_to_mel_htk(f):
    return 2595.0 * np.log10(1.0 + np.asarray(f, dtype=np.float64) / 700.0)


def _mel_to_hz_htk(m):
    return 700.0 * (10.0 ** (np.asarray(m, dtype=np.float64) / 2595.0) - 1.0)


def htk_mel_fbanks(n_freqs: int, f_min: float, f_max: float, n_mels: int, sample_rate: int) -> np.ndarray:
    """torchaudio.functional.melscale_fbanks(norm=None, mel_scale='htk') -> (n_freqs, n_mels).

    all_freqs = linspace(0, sr//2, n_freqs); f_pts = mel_to_hz(linspace(mel(f_min), mel(f_max), n_mels+2));
    triangular filter = max(0, min(down_slope, up_slope)).
    """
    all_freqs = np.linspace(0.0, float(sample_rate // 2), n_freqs)
    m_pts = np.linspace(_hz_to_mel_htk(f_min), _hz_to_mel_htk(f_max), n_mels + 2)
    f_pts = _mel_to_hz_htk(m_pts)
    f_diff = f_pts[1:] - f_pts[:-1]
    slopes = f_pts[None, :] - all_freqs[:, None]
    down = (-1.0 * slopes[:, :-2]) / f_diff[:-1]
    up = slopes[:, 2:] / f_diff[1:]
    return np.maximum(0.0, np.minimum(down, up))


def _hz_to_mel_slaney(f):
    f = np.asarray(f, dtype=np.float64)
    f_sp = 200.0 / 3.0
    mels = f / f_sp
    min_log_hz = 1000.0
    min_log_mel = min_log_hz / f_sp
    logstep = math.log(6.4) / 27.0
    return np.where(f >= min_log_hz, min_log_mel + np.log(np.maximum(f, 1e-30) / min_log_hz) / logstep, mels)


def _mel_to_hz_slaney(m):
    m = np.asarray(m, dtype=np.float64)
    f_sp = 200.0 / 3.0
    freqs = f_sp * m
    min_log_hz = 1000.0
    min_log_mel = min_log_hz / f_sp
    logstep = math.log(6.4) / 27.0
    return np.where(m >= min_log_mel, min_log_hz * np.exp(logstep * (m - min_log_mel)), freqs)


def slaney_mel_fbanks(sample_rate: int, n_fft: int, n_mels: int = 128, fmin: float = 0.0, fmax: float | None = None) -> np.ndarray:
    """librosa.filters.mel(htk=False, norm='slaney', dtype=float32) -> (n_freqs, n_mels) (transposed)."""
    if fmax is None:
        fmax = sample_rate / 2.0
    fftfreqs = np.fft.rfftfreq(n=n_fft, d=1.0 / sample_rate)
    mel_f = _mel_to_hz_slaney(np.linspace(_hz_to_mel_slaney(fmin), _hz_to_mel_slaney(fmax), n_mels + 2))
    fdiff = np.diff(mel_f)
    ramps = mel_f[:, None] - fftfreqs[None, :]
    w = np.zeros((n_mels, fftfreqs.size), dtype=np.float64)
    for i in range(n_mels):
        lower = -ramps[i] / fdiff[i]
        upper = ramps[i + 2] / fdiff[i + 1]
        w[i] = np.maximum(0.0, np.minimum(lower, upper))
    enorm = 2.0 / (mel_f[2:n_mels + 2] - mel_f[:n_mels])
    w *= enorm[:, None]
    # librosa stores the basis as float32 (its default dtype); keep that rounding.
    return w.astype(np.float32).astype(np.float64).T


def dct_ortho(n_mfcc: int, n_mels: int) -> np.ndarray:
    """torchaudio.functional.create_dct(n_mfcc, n_mels, norm='ortho') -> (n_mels, n_mfcc).

    Identical to scipy DCT-II norm='ortho' restricted to the first n_mfcc outputs.
    """
    n = np.arange(n_mels, dtype=np.float64)
    k = np.arange(n_mfcc, dtype=np.float64)[:, None]
    d = np.cos(math.pi / n_mels * (n + 0.5) * k)
    d[0] *= 1.0 / math.sqrt(2.0)
    d *= math.sqrt(2.0 / n_mels)
    return d.T


# ----------------------------------------------------------------------------- stages
def n_frames(length: int, n_fft: int, hop: int) -> int:
    """Frame count with center=True: 1 + (L + 2*(n_fft//2) - n_fft) // hop."""
    return 1 + (length + 2 * (n_fft // 2) - n_fft) // hop


def stft_power(wave: np.ndarray, n_fft: int, hop: int, pad_mode: str = "reflect") -> np.ndarray:
    """|STFT|^2, onesided, center=True, periodic Hann.  wave (B, L) -> (B, n_fft//2+1, T) float64."""
    wave = np.asarray(wave, dtype=np.float64)
    if wave.ndim == 1:
        wave = wave[None]
    pad = n_fft // 2
    mode = {"reflect": "reflect", "constant": "constant"}[pad_mode]
    xp = np.pad(wave, ((0, 0), (pad, pad)), mode=mode)
    T = n_frames(wave.shape[1], n_fft, hop)
    idx = np.arange(T)[:, None] * hop + np.arange(n_fft)[None, :]
    frames = xp[:, idx] * hann_periodic(n_fft)[None, None, :]  # (B, T, n_fft)
    spec = np.fft.rfft(frames, axis=-1)
    p = spec.real ** 2 + spec.imag ** 2
    return np.transpose(p, (0, 2, 1))


def amplitude_to_db(x: np.ndarray, top_db: float = 80.0, amin: float = 1e-10) -> np.ndarray:
    """AmplitudeToDB('power') / librosa power_to_db(ref=1): x (B, n_mels, T), max per utterance."""
    db = 10.0 * np.log10(np.maximum(x, amin))
    if top_db is not None:
        mx = db.reshape(db.shape[0], -1).max(axis=1)
        db = np.maximum(db, (mx - top_db)[:, None, None])
    return db


def mfcc_core(wave2d: np.ndarray, sample_rate: int, n_mfcc: int, n_fft: int, hop: int,
              mel: str = "htk", pad_mode: str = "reflect", n_mels: int = 128, top_db: float = 80.0) -> np.ndarray:
    """(B, L) -> (B, n_mfcc, T) float64 for either front end."""
    p = stft_power(wave2d, n_fft, hop, pad_mode)
    n_freqs = n_fft // 2 + 1
    if mel == "htk":
        fb = htk_mel_fbanks(n_freqs, 0.0, float(sample_rate // 2), n_mels, sample_rate)
    elif mel == "slaney":
        fb = slaney_mel_fbanks(sample_rate, n_fft, n_mels)
    else:
        raise ValueError(f"unknown mel scale {mel!r}")
    melspec = np.einsum("bft,fm->bmt", p, fb, optimize=True)
    db = amplitude_to_db(melspec, top_db=top_db)
    return np.einsum("bmt,mc->bct", db, dct_ortho(n_mfcc, n_mels), optimize=True)


def mfcc_torchaudio(waveform, sample_rate: int, n_mfcc: int, n_fft: int, hop_length: int) -> np.ndarray:
    """Reference ``MFCC()`` (prepare_dataset.py:35-47): (L,) -> (n_mfcc, T); (N,1,L) -> (N,1,n_mfcc,T)."""
    w = np.asarray(waveform, dtype=np.float64)
    if w.ndim == 1:
        return mfcc_core(w[None], sample_rate, n_mfcc, n_fft, hop_length)[0]
    if w.ndim == 3 and w.shape[1] == 1:
        return mfcc_core(w[:, 0], sample_rate, n_mfcc, n_fft, hop_length)[:, None]
    raise ValueError("oracle MFCC supports (L,) and (N,1,L) inputs (the reference's two call shapes)")


def mfcc_librosa(waveform, sample_rate: int, n_mfcc: int, n_fft: int = 2048, hop_length: int = 512,
                 pad_mode: str = "constant") -> np.ndarray:
    """Reference ``librosa_MFCC()`` (utils/daba_selection_tools.py:16-22): (L,) -> (n_mfcc, T)."""
    w = np.asarray(waveform, dtype=np.float64)
    return mfcc_core(w[None], sample_rate, n_mfcc, n_fft, hop_length, mel="slaney", pad_mode=pad_mode)[0]


def mfcc_model_input(wave2d, sample_rate, n_mfcc, n_fft, hop, mel="htk", pad_mode="reflect") -> np.ndarray:
    """What the callers hand the model: ``MFCC(..).numpy().T[np.newaxis]`` -> (B, 1, T, n_mfcc)."""
    c = mfcc_core(wave2d, sample_rate, n_mfcc, n_fft, hop, mel=mel, pad_mode=pad_mode)
    return np.transpose(c, (0, 2, 1))[:, None]
