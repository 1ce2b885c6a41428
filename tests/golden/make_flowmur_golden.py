#!/usr/bin/env python3
"""FlowMur trigger-optimisation golden vectors: torch float64 AUTOGRAD of the reference loop.

Run in the build container (where /root/reference exists):
    python tests/golden/make_flowmur_golden.py      -> tests/golden/flowmur_golden.npz

The frozen model is the reference's own ``utils.models.smallcnn`` (imported from
/root/reference, eval mode like the EarlyStoppingModel checkpoint, float64).  The rest of
utils/flowmur_generate_trigger.py:64-118 cannot be imported here (it imports torchaudio), so
this script restates it line by line with torch ops:
  * deploy_trigger_to_waveform (:49-62) with the positions pinned;
  * clamp(-1, 1) (:92);
  * torchaudio T.MFCC(16000, 13, n_fft 2048, hop 512): torch.stft(center, reflect, periodic
    Hann) -> |.|^2 -> HTK mel (oracle.mfcc tables) -> AmplitudeToDB's code path
    (clamp_min(amin), 10 log10, torch.max against amax - top_db over the packed dims) ->
    ortho DCT matmul;
  * CrossEntropyLoss, the accumulated ``loss = loss + criterion(...)`` with
    ``backward(retain_graph=True)``, Adam(lr 1e-3), ``trigger.data = clamp(.., -0.2, 0.2)``.
Autograd differentiates the whole chain, so the fixture pins the hand-derived adjoints of
oracle/flowmur.py (and, through it, libabd's backward kernels) and the loop's
gradient-accumulation semantics.  Only outputs are stored; inputs regenerate from seeds
(tests/golden_inputs.py flowmur_inputs).
"""
from __future__ import annotations

import os
import sys

import numpy as np

REF = os.environ.get("ABD_REFERENCE", "/root/reference")
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.dont_write_bytecode = True
sys.path.insert(0, REF)
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(1, ROOT)

import torch  # noqa: E402

from golden_inputs import FLOWMUR, flowmur_inputs  # noqa: E402
from oracle import mfcc as om  # noqa: E402

import utils.models as ref_models  # noqa: E402

D = torch.float64


def deploy(waveforms, trigger, positions):
    """utils/flowmur_generate_trigger.py:49-62 with position i = positions[i] (random.randint there)."""
    waveforms_rms = torch.linalg.norm(waveforms, dim=2)
    trigger_rms = torch.linalg.norm(trigger.clone(), dim=1)
    scale = 10 ** (30 / 20) * (trigger_rms / waveforms_rms)
    new_waveforms = torch.tensor([], dtype=D)
    for i, wav in enumerate(waveforms):
        position = int(positions[i])
        befo_tr = scale[i] * wav[0][0:position] / (scale[i] + 1)
        in_tr = (scale[i] * wav[0][position:position + trigger.shape[1]] + trigger[0]) / (scale[i] + 1)
        af_tr = scale[i] * wav[0][position + trigger.shape[1]:] / (scale[i] + 1)
        new_wav = torch.cat([befo_tr, in_tr, af_tr]).unsqueeze(dim=0).unsqueeze(dim=0)
        new_waveforms = torch.cat((new_waveforms, new_wav), dim=0)
    return new_waveforms


class TorchMFCC:
    """torchaudio.transforms.MFCC(16000, 13, melkwargs={n_fft 2048, hop 512}) restated with torch ops."""

    def __init__(self, sr=16000, n_mfcc=13, n_fft=2048, hop=512, n_mels=128, top_db=80.0):
        self.n_fft, self.hop, self.top_db = n_fft, hop, top_db
        self.window = torch.hann_window(n_fft, periodic=True, dtype=D)
        self.fb = torch.tensor(om.htk_mel_fbanks(n_fft // 2 + 1, 0.0, float(sr // 2), n_mels, sr), dtype=D)
        self.dct = torch.tensor(om.dct_ortho(n_mfcc, n_mels), dtype=D)

    def __call__(self, wave):  # (B, 1, L) -> (B, 1, n_mfcc, T)
        shape = wave.shape
        spec = torch.stft(wave.reshape(-1, shape[-1]), self.n_fft, self.hop, win_length=self.n_fft,
                          window=self.window, center=True, pad_mode="reflect", normalized=False, onesided=True,
                          return_complex=True)
        power = spec.abs().pow(2.0)
        power = power.reshape(shape[:-1] + power.shape[-2:])                     # (B, 1, NF, T)
        mel = torch.matmul(power.transpose(-1, -2), self.fb).transpose(-1, -2)  # (B, 1, n_mels, T)
        x_db = 10.0 * torch.log10(torch.clamp(mel, min=1e-10))
        x_db = x_db - 10.0 * np.log10(max(1e-10, 1.0))
        s = x_db.size()
        packed = s[-3] if x_db.dim() > 2 else 1
        x_db = x_db.reshape(-1, packed, s[-2], s[-1])
        x_db = torch.max(x_db, (x_db.amax(dim=(-3, -2, -1)) - self.top_db).view(-1, 1, 1, 1))
        x_db = x_db.reshape(s)
        return torch.matmul(x_db.transpose(-1, -2), self.dct).transpose(-1, -2)


def main():
    torch.set_num_threads(4)
    c = FLOWMUR
    waves, pos, labels, state = flowmur_inputs()
    model = ref_models.smallcnn(c["K"], c["lf"])
    model.load_state_dict({k: torch.tensor(v) for k, v in state.items()})
    model = model.double().eval()
    for p in model.parameters():
        p.requires_grad = False
    mfcc = TorchMFCC()
    criterion = torch.nn.CrossEntropyLoss()
    trigger = torch.autograd.Variable(torch.ones((1, c["Lt"]), dtype=D) * 0.1, requires_grad=True)
    optimizer = torch.optim.Adam(params=[trigger], lr=0.001)
    y = torch.tensor(labels)
    out = {}
    traj, losses = [], []
    for epoch in range(c["epochs"]):
        loss = 0
        for bi in range(c["n_batches"]):
            w = torch.tensor(waves[bi * c["B"]:(bi + 1) * c["B"]], dtype=D)[:, None]
            new = deploy(w, trigger, pos[epoch, bi])
            wc = torch.clamp(new, -1, 1)
            feats = mfcc(wc).permute(0, 1, 3, 2)
            pred = model.forward(feats)
            batch_loss = criterion(pred, y)
            loss = loss + batch_loss
            optimizer.zero_grad()
            loss.backward(retain_graph=True)
            if epoch == 0 and bi == 0:
                out["grad0"] = trigger.grad.detach().numpy()[0].copy()
                out["feats0"] = feats.detach().numpy()
                out["logp0"] = pred.detach().numpy()
                out["loss0"] = np.array(float(batch_loss))
            optimizer.step()
            trigger.data = torch.clamp(trigger.data, -0.2, 0.2)
            traj.append(trigger.detach().numpy()[0].copy())
        losses.append(float(loss))
    out["traj"] = np.stack(traj)
    out["epoch_loss"] = np.array(losses)
    np.savez_compressed(os.path.join(HERE, "flowmur_golden.npz"), **out)
    print("wrote flowmur_golden.npz:", {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
