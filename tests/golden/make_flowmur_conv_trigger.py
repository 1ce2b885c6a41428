#!/usr/bin/env python3
"""The FlowMur trigger of the flowmur convergence fixture (tests/golden/flowmur_conv_trigger.npy).

flowmur.py:53-67 loads a pretrained surrogate (smallcnn_10_2.pkl) and an optimised trigger
(sp_trigger300.npy) that the reference does not ship.  This script makes both the way the
reference's commented-out calls would, on the convergence fixture's own clean clips:

* surrogate: the reference's ``utils.models.smallcnn(10, 224)`` trained with its
  ``utils.training_tools.clean_train`` (pretrain_model, flowmur_generate_trigger.py:15-47: 80/20
  split with random_state 35, batch 256, Adam lr 1e-4 -- a fixed epoch count instead of early
  stopping over 1000 epochs);
* trigger: generate_trigger (:64-118) -- ones * 0.1, Adam(lr 1e-3) on the trigger, the SNR-30 mix of
  deploy_trigger_to_waveform (:49-62), clamp(-1, 1), MFCC(16000, 13, 2048, 512) (torchaudio's
  T.MFCC restated in torch, oracle/torch_ref.py: differentiable), the frozen surrogate, CE towards
  label 2, clamp +-0.2 -- with the loss of each batch on its own (the reference accumulates the
  graph across batches) and a fixed, small epoch count.

Run in the build container (imports /root/reference):  python tests/golden/make_flowmur_conv_trigger.py
"""
from __future__ import annotations

import os
import random
import sys

import numpy as np

REF = os.environ.get("ABD_REFERENCE", "/root/reference")
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.dont_write_bytecode = True
sys.path.insert(0, REF)
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from golden_inputs import CONV_CFGS  # noqa: E402
from abd_amd import synth  # noqa: E402
from oracle import torch_ref  # noqa: E402
import utils.models as ref_models  # noqa: E402
import utils.training_tools as ref_tt  # noqa: E402

SURROGATE_EPOCHS = 6
TRIGGER_EPOCHS = 12


def deploy(waves, trigger, rnd):
    """deploy_trigger_to_waveform (flowmur_generate_trigger.py:49-62), batched."""
    wr = torch.linalg.norm(waves, dim=2)                     # (B, 1)
    tr = torch.linalg.norm(trigger, dim=1)                   # (1,)
    s = (10 ** (30 / 20)) * (tr / wr)                        # (B, 1)
    out = []
    for i in range(waves.shape[0]):
        p = rnd.randint(0, waves.shape[2] - trigger.shape[1])
        w = waves[i, 0]
        out.append(torch.cat([s[i] * w[:p] / (s[i] + 1), (s[i] * w[p:p + trigger.shape[1]] + trigger[0]) / (s[i] + 1),
                              s[i] * w[p + trigger.shape[1]:] / (s[i] + 1)]))
    return torch.stack(out)[:, None]


def main():
    c = CONV_CFGS["flowmur"]
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    waves, labels = synth.make_clips_np(c["n_train"] + c["n_test"], c["sr"], c["L"], c["K"], seed=c["clip_seed"])
    ntr = c["n_train"]
    w = torch.from_numpy(waves[:ntr].copy())
    y = torch.from_numpy(labels[:ntr].copy())
    feat = torch_ref.MfccCPU(c["sr"], c["n_mfcc"], c["n_fft"], c["hop"])
    x = torch.cat([feat(w[s:s + 256]) for s in range(0, ntr, 256)])
    # pretrain_model: 80/20 split (random_state 35), batch 256, Adam 1e-4
    from sklearn.model_selection import train_test_split
    torch.manual_seed(77)
    random.seed(77)
    xt, xv, yt, yv = train_test_split(x, y, test_size=0.2, random_state=35)
    tl = torch.utils.data.DataLoader(torch.utils.data.TensorDataset(xt, yt), batch_size=256, shuffle=True)
    vl = torch.utils.data.DataLoader(torch.utils.data.TensorDataset(xv, yv), batch_size=256, shuffle=True)
    m = ref_models.smallcnn(c["K"], c["lf"])
    opt = torch.optim.Adam(m.parameters(), lr=1e-4)
    crit = torch.nn.CrossEntropyLoss()
    for e in range(SURROGATE_EPOCHS):
        tl_, ta = ref_tt.clean_train(m, tl, torch.device("cpu"), opt, crit)
        vl_, va = ref_tt.clean_test(m, torch.device("cpu"), vl, crit)
        print(f"surrogate epoch {e + 1}: train {tl_:.4f}/{ta:.2f}  val {vl_:.4f}/{va:.2f}", flush=True)
    m.eval()
    for p in m.parameters():
        p.requires_grad = False
    # generate_trigger: 5000 (here: every) training clips labelled 2, batch 256, shuffled
    trig = torch.full((1, c["Lt"]), 0.1, requires_grad=True)
    topt = torch.optim.Adam([trig], lr=1e-3)
    rnd = random.Random(91)
    ds = torch.utils.data.DataLoader(torch.utils.data.TensorDataset(w[:, None], torch.full((ntr,), 2)),
                                     batch_size=256, shuffle=True)
    for e in range(TRIGGER_EPOCHS):
        tot = 0.0
        for wb, lb in ds:
            xm = torch.clamp(deploy(wb, trig, rnd), -1, 1)
            loss = crit(m(feat(xm[:, 0])), lb)
            topt.zero_grad()
            loss.backward()
            topt.step()
            with torch.no_grad():
                trig.clamp_(-0.2, 0.2)
            tot += float(loss)
        print(f"trigger epoch {e + 1}: mean CE to label 2 {tot / len(ds):.4f}", flush=True)
    out = trig.detach()[0].numpy().astype(np.float32)
    np.save(os.path.join(HERE, "flowmur_conv_trigger.npy"), out)
    print("wrote flowmur_conv_trigger.npy", out.shape, float(np.abs(out).max()))


if __name__ == "__main__":
    main()
