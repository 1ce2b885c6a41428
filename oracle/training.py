"""Oracle (test infrastructure): train()/test() bookkeeping restated (utils/training_tools.py:52-134)."""
from __future__ import annotations

import numpy as np

from .smallcnn import SmallCNN


def train_epoch(model: SmallCNN, batches, masks, lr=1e-4):
    """batches: list of (mfcc (B,1,H,W), label (B,), indicator (B,)); masks: list of (mask1, mask2).

    Returns (train_loss, train_mix_acc, train_asr) exactly as train() (:52-85) computes them:
    mean of per-batch mean losses, 100*correct/total, 100*asr_correct/poison_total.
    """
    running, correct, total, asr_c, ptotal = 0.0, 0, 0, 0, 0
    for (x, y, ind), (m1, m2) in zip(batches, masks):
        out, loss, _ = model.train_step(x, y, m1, m2, lr=lr)
        running += float(loss)
        pred = out.argmax(axis=1)
        total += len(y)
        correct += int((pred == y).sum())
        sel = np.asarray(ind) == 1
        ptotal += int(sel.sum())
        asr_c += int((pred[sel] == np.asarray(y)[sel]).sum())
    return running / len(batches), 100.0 * correct / total, 100 * asr_c / ptotal


def test(model: SmallCNN, clean_batches, bd_batches):
    """test() (:87-134): returns (clean_acc, asr, clean_loss, bd_loss)."""
    cc, ct, cl = 0, 0, 0.0
    for x, y in clean_batches:
        out = model.forward_eval(x)
        cl += float(SmallCNN.ce_loss_and_grad(out, np.asarray(y))[0])
        pred = out.argmax(axis=1)
        ct += len(y)
        cc += int((pred == y).sum())
    ac, pt, bl = 0, 0, 0.0
    for x, y, ind in bd_batches:
        out = model.forward_eval(x)
        bl += float(SmallCNN.ce_loss_and_grad(out, np.asarray(y))[0])
        pred = out.argmax(axis=1)
        sel = np.asarray(ind) == 1
        pt += int(sel.sum())
        ac += int((pred[sel] == np.asarray(y)[sel]).sum())
    return 100 * cc / ct, 100 * ac / pt, cl / len(clean_batches), bl / len(bd_batches)
