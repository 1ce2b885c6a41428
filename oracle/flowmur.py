"""Oracle (test infrastructure): FlowMur trigger-gradient chain restated in float64 numpy.

Follows reference ``utils/flowmur_generate_trigger.py``:
  * ``deploy_trigger_to_waveform`` (:49-62): s = 10^(30/20) |t| / |w|,
    x = (s w + t)/(s+1) inside [p, p+Lt), s w/(s+1) outside;
  * ``torch.clamp(new_waveforms, -1, 1)`` (:92);
  * ``T.MFCC(16000, 13, melkwargs={n_fft 2048, hop 512})`` (:65-74, :93), i.e. the
    torchaudio MFCC restated in ``oracle.mfcc`` (reflect pad, Hann, power 2, HTK mel,
    AmplitudeToDB(top_db=80) per utterance, ortho DCT);
  * the frozen benign model in eval mode (:98; it is the checkpoint EarlyStoppingModel
    writes right after clean_test(), training_tools.py:49/160) and CrossEntropyLoss (:101);
  * ``loss.backward()`` to the trigger (:103), including the path through s(|t|).
Backward rules follow torch autograd: clamp passes the gradient for -1 <= y <= 1,
``torch.maximum`` gives a tie half the gradient, ``amax`` splits the gradient evenly over
the maxima, ``clamp_min(amin)`` passes it for x >= amin.

The adjoints are derived by hand; ``tests/golden/make_flowmur_golden.py`` pins them against
torch float64 autograd of the same chain (tests/golden/flowmur_golden.npz).
"""
from __future__ import annotations

import math

import numpy as np

from . import mfcc as om

SNR_GAIN = 10.0 ** (30.0 / 20.0)
AMIN = 1e-10


def deploy(w, t, pos):
    """(B, L) clean waves, (Lt,) trigger, (B,) positions -> (mixed (B, L) before the clamp, s (B,))."""
    w = np.asarray(w, np.float64)
    t = np.asarray(t, np.float64).reshape(-1)
    tn = math.sqrt(float(t @ t))
    s = SNR_GAIN * tn / np.sqrt((w * w).sum(axis=1))
    x = s[:, None] * w
    tin = np.zeros_like(w)
    for i, p in enumerate(pos):
        tin[i, int(p):int(p) + t.size] = t
    return (x + tin) / (s[:, None] + 1.0), s, tin


def mfcc_forward(x, sample_rate=16000, n_mfcc=13, n_fft=2048, hop=512, n_mels=128, top_db=80.0):
    """(B, L) -> (model input (B, 1, T, n_mfcc), cache) with every intermediate the backward needs."""
    x = np.asarray(x, np.float64)
    pad = n_fft // 2
    xp = np.pad(x, ((0, 0), (pad, pad)), mode="reflect")
    T = om.n_frames(x.shape[1], n_fft, hop)
    idx = np.arange(T)[:, None] * hop + np.arange(n_fft)[None, :]
    win = om.hann_periodic(n_fft)
    X = np.fft.rfft(xp[:, idx] * win, axis=-1)                  # (B, T, NF)
    P = X.real ** 2 + X.imag ** 2
    fb = om.htk_mel_fbanks(n_fft // 2 + 1, 0.0, float(sample_rate // 2), n_mels, sample_rate)
    mel = np.einsum("btf,fm->btm", P, fb)                       # (B, T, n_mels)
    db = 10.0 * np.log10(np.maximum(mel, AMIN))
    mx = db.reshape(db.shape[0], -1).max(axis=1)
    thr = mx - top_db
    dbc = np.maximum(db, thr[:, None, None])
    dct = om.dct_ortho(n_mfcc, n_mels)                          # (n_mels, n_mfcc)
    out = np.einsum("btm,mc->btc", dbc, dct)[:, None]
    cache = dict(L=x.shape[1], pad=pad, T=T, hop=hop, n_fft=n_fft, win=win, X=X, fb=fb, mel=mel, db=db, mx=mx,
                 thr=thr, dct=dct)
    return out, cache


def mfcc_backward(dout, c):
    """d loss / d (B, 1, T, n_mfcc) -> d loss / d x (B, L)."""
    d = np.einsum("btc,mc->btm", np.asarray(dout, np.float64)[:, 0], c["dct"])
    db, thr, mx = c["db"], c["thr"][:, None, None], c["mx"][:, None, None]
    gt, tie, lt = db > thr, db == thr, db < thr
    g = d * gt + 0.5 * d * tie
    mass = (d * lt).sum(axis=(1, 2)) + 0.5 * (d * tie).sum(axis=(1, 2))
    ismax = db == mx
    g = g + ismax * (mass / ismax.sum(axis=(1, 2)))[:, None, None]
    mel = c["mel"]
    dmel = np.where(mel >= AMIN, g * (10.0 / math.log(10.0)) / np.maximum(mel, AMIN), 0.0)
    dP = np.einsum("btm,fm->btf", dmel, c["fb"])               # (B, T, NF)
    Y = dP * np.conj(c["X"])
    N = c["n_fft"]
    H = np.zeros(Y.shape[:2] + (N,), np.complex128)             # Hermitian extension, DC / Nyquist doubled
    H[..., :N // 2 + 1] = Y
    H[..., N // 2 + 1:] = np.conj(Y[..., 1:N // 2][..., ::-1])
    H[..., 0] *= 2.0
    H[..., N // 2] *= 2.0
    gfr = np.fft.fft(H, axis=-1).real * c["win"]                # d loss / d frame sample
    B, T = gfr.shape[:2]
    L, pad, hop = c["L"], c["pad"], c["hop"]
    dpad = np.zeros((B, L + 2 * pad))
    for t in range(T):
        dpad[:, t * hop:t * hop + N] += gfr[:, t]
    dx = dpad[:, pad:pad + L].copy()
    dx[:, 1:pad + 1] += dpad[:, :pad][:, ::-1]                  # left reflection: padded[i] = x[pad - i]
    dx[:, L - 1 - pad:L - 1] += dpad[:, pad + L:][:, ::-1]      # right: padded[pad+L+j] = x[L-2-j]
    return dx


def deploy_backward(dxc, w, t, s, tin, pos, x_mixed, clamp=True):
    """d loss / d clamp(deploy(w, t)) -> d loss / d t (through the window and through s(|t|))."""
    t = np.asarray(t, np.float64).reshape(-1)
    dx = np.asarray(dxc, np.float64)
    if clamp:
        dx = dx * ((x_mixed >= -1.0) & (x_mixed <= 1.0))
    w = np.asarray(w, np.float64)
    dt = np.zeros_like(t)
    for i, p in enumerate(pos):
        dt += dx[i, int(p):int(p) + t.size] / (s[i] + 1.0)
    dS = (dx * (w - tin)).sum(axis=1) / (s + 1.0) ** 2
    dt += t * float((s * dS).sum()) / float(t @ t)
    return dt


def trigger_grad(model, w, t, pos, labels, clamp=True, **mfcc_kw):
    """One batch of utils/flowmur_generate_trigger.py:91-103: (loss, d loss / d t, model input, log-probs)."""
    xm, s, tin = deploy(w, t, pos)
    xc = np.clip(xm, -1.0, 1.0) if clamp else xm
    feats, cache = mfcc_forward(xc, **mfcc_kw)
    out, loss, dfeat = model.input_grad_eval(feats, labels)
    dxc = mfcc_backward(dfeat, cache)
    return loss, deploy_backward(dxc, w, t, s, tin, pos, xm, clamp=clamp), feats, out


def optimise(model, batches, trigger_length, epochs, lr=1e-3, bound=0.2, init=0.1):
    """generate_trigger's loop (:79-105) over fixed batches [(w, labels, positions per epoch)]:
    the loss graph accumulates over an epoch, so step j uses sum_{i<=j} grad_i, then Adam, then clamp."""
    t = np.full(trigger_length, init)
    m = np.zeros_like(t)
    v = np.zeros_like(t)
    step = 0
    traj = []
    for e in range(epochs):
        acc = np.zeros_like(t)
        for w, labels, pos in batches[e]:
            _, g, _, _ = trigger_grad(model, w, t, pos, labels)
            acc = acc + g
            step += 1
            m = m + (1 - 0.9) * (acc - m)
            v = v * 0.999 + (1 - 0.999) * acc * acc
            denom = np.sqrt(v) / math.sqrt(1 - 0.999 ** step) + 1e-8
            t = t - lr / (1 - 0.9 ** step) * m / denom
            t = np.clip(t, -bound, bound)
            traj.append(t.copy())
    return np.stack(traj)
