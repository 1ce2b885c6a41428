"""DABA selection restated in float64 numpy -- TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

utils/daba_selection_tools.py:
  * one_sotamax_entropy (:68-87): librosa MFCC of the clip as read by soundfile (int16/32768),
    ``mfcc[:, :32]`` or ``np.pad(..., constant_values=-200)`` to 32 frames, a batch-1 forward of
    the train-mode model (BatchNorm over that one clip, dropout active), F.softmax, calc_ent.
  * calc_ent (:53-65): -sum p log2 p.
  * cross_entropy (:67-68): sum nan_to_num(-y log a - (1-y) log(1-a)).
  * Inf_cross_entropy (:113-139): single_trigger_injection_db(host, trigger, po_db) -> wav ->
    soundfile float, then cross_entropy(softmax(trigger), softmax(poisoned)).
The forward is pinned by tests/golden/make_daba_golden.py (the reference's smallcnn run at
batch 1 in train mode); calc_ent / cross_entropy / the pad rule are restated (their module
imports pydub and librosa at the top, which the image lacks: parity unpinned for those lines).
"""
from __future__ import annotations

import math

import numpy as np

from . import mfcc as om
from . import triggers as ot

N_FRAMES = 32


def selection_input(clip_int16, sample_rate=16000, n_mfcc=40):
    """(1, 1, 32, 40) model input of one clip (daba_selection_tools.py:69-80)."""
    w = np.asarray(clip_int16, dtype=np.float64) / 32768.0
    m = om.mfcc_librosa(w, sample_rate, n_mfcc)
    if m.shape[1] > N_FRAMES:
        m = m[:, :N_FRAMES]
    else:
        m = np.pad(m, ((0, 0), (0, N_FRAMES - m.shape[1])), mode="constant", constant_values=-200)
    return m.T[None, None]


def softmax(logp):
    z = np.asarray(logp, dtype=np.float64)
    e = np.exp(z - z.max(axis=-1, keepdims=True))
    return e / e.sum(axis=-1, keepdims=True)


def calc_ent(p):
    return -float(sum(x * math.log2(x) for x in np.asarray(p, dtype=np.float64)))


def cross_entropy(a, y):
    a = np.asarray(a, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64)
    with np.errstate(divide="ignore", invalid="ignore"):
        return float(np.sum(np.nan_to_num(-y * np.log(a) - (1 - y) * np.log(1 - a))))


def per_utterance_forward(net, x, mask1, mask2):
    """Batch-1 train-mode forwards, one per row (net: oracle.smallcnn.SmallCNN)."""
    out = []
    for i in range(x.shape[0]):
        lp, _ = net.forward_train(x[i:i + 1], mask1[i:i + 1], mask2[i:i + 1])
        out.append(lp[0])
    return np.stack(out)


def poisoned_clip(host_int16, trig_int16, po_db=-20):
    return ot.single_trigger_injection_db(host_int16, trig_int16, po_db)
