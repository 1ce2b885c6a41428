"""Oracle (test infrastructure): the reference CPU path restated in torch float32.

Where ``oracle.mfcc`` / ``oracle.smallcnn`` restate the path in float64 numpy (the
checker), this module restates it with the same torch CPU ops the reference runs,
in the reference's own precision.  It serves two roles and nothing else:

* ``bench.py``'s ``cpu_baseline`` leg: the reference CPU path timed on the GPU
  box's host cores (torch/numpy restatement at the bench batch);
* fast host-side features for the multi-epoch convergence fixtures
  (``tests/golden/make_convergence.py``) and their GPU replay tests.

It is never imported by the product (``audio-backdoor-attack_amd/``).

Restated algorithms (reference file:line -> third-party call it makes):

* ``mfcc``: ``prepare_dataset.py:35-47`` -> torchaudio ``T.MFCC(sample_rate,
  n_mfcc, melkwargs={n_fft, hop_length})`` with torchaudio's defaults: periodic
  Hann window of n_fft, ``torch.stft(center=True, pad_mode='reflect',
  onesided=True)``, ``abs().pow(2)``, HTK mel filterbank (norm None, f_min 0,
  f_max sr//2, 128 mels) built in float32 like ``melscale_fbanks``,
  ``AmplitudeToDB('power', top_db=80)`` (amin 1e-10, max per utterance), DCT-II
  ``create_dct(norm='ortho')``; output ``.T[np.newaxis]`` -> (N, 1, T, n_mfcc).
* ``SmallCNN``: ``utils/models.py:17-65`` (same submodules and parameter names,
  so reference state_dicts load unchanged).
* ``train_step``: one iteration of ``utils/training_tools.py:60-79``.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as Fn


def _hz_to_mel_htk(f: float) -> float:
    return 2595.0 * math.log10(1.0 + f / 700.0)


def htk_fbanks(n_freqs: int, sample_rate: int, n_mels: int = 128) -> torch.Tensor:
    """torchaudio.functional.melscale_fbanks(n_freqs, 0, sr//2, n_mels, sr, norm=None, 'htk'): (n_freqs, n_mels)
    in float32, the precision torchaudio builds it in."""
    all_freqs = torch.linspace(0, sample_rate // 2, n_freqs)
    m_pts = torch.linspace(_hz_to_mel_htk(0.0), _hz_to_mel_htk(float(sample_rate // 2)), n_mels + 2)
    f_pts = 700.0 * (10.0 ** (m_pts / 2595.0) - 1.0)
    f_diff = f_pts[1:] - f_pts[:-1]
    slopes = f_pts.unsqueeze(0) - all_freqs.unsqueeze(1)
    down = (-1.0 * slopes[:, :-2]) / f_diff[:-1]
    up = slopes[:, 2:] / f_diff[1:]
    return torch.max(torch.zeros(1), torch.min(down, up))


def dct_ortho(n_mfcc: int, n_mels: int) -> torch.Tensor:
    """torchaudio.functional.create_dct(n_mfcc, n_mels, 'ortho'): (n_mels, n_mfcc) float32."""
    n = torch.arange(float(n_mels))
    k = torch.arange(float(n_mfcc)).unsqueeze(1)
    d = torch.cos(math.pi / float(n_mels) * (n + 0.5) * k)
    d[0] *= 1.0 / math.sqrt(2.0)
    d *= math.sqrt(2.0 / float(n_mels))
    return d.t()


class MfccCPU:
    """Tables for one (sr, n_mfcc, n_fft, hop) configuration; call on (N, L) float32 CPU waves."""

    def __init__(self, sample_rate: int, n_mfcc: int, n_fft: int, hop_length: int, n_mels: int = 128,
                 top_db: float = 80.0):
        self.sr, self.n_mfcc, self.n_fft, self.hop = sample_rate, n_mfcc, n_fft, hop_length
        self.top_db = top_db
        self.window = torch.hann_window(n_fft)
        self.fb = htk_fbanks(n_fft // 2 + 1, sample_rate, n_mels)
        self.dct = dct_ortho(n_mfcc, n_mels)

    def __call__(self, waves: torch.Tensor) -> torch.Tensor:
        x = waves.reshape(-1, waves.shape[-1]).float()
        spec = torch.stft(x, self.n_fft, self.hop, self.n_fft, self.window, center=True, pad_mode="reflect",
                          normalized=False, onesided=True, return_complex=True)
        power = spec.abs().pow(2.0)                                         # (N, F, T)
        mel = torch.matmul(power.transpose(-1, -2), self.fb).transpose(-1, -2)   # (N, n_mels, T)
        db = 10.0 * torch.log10(torch.clamp(mel, min=1e-10))
        mx = db.amax(dim=(-2, -1))                                          # per utterance
        db = torch.max(db, (mx - self.top_db).view(-1, 1, 1))
        return torch.matmul(db.transpose(-1, -2), self.dct).unsqueeze(1)    # (N, 1, T, n_mfcc)


def mfcc(waves: torch.Tensor, sample_rate: int, n_mfcc: int, n_fft: int, hop_length: int,
         chunk: int = 256) -> torch.Tensor:
    """(N, L) float32 -> (N, 1, T, n_mfcc): the reference's per-clip ``MFCC(..).numpy().T[np.newaxis]``."""
    f = MfccCPU(sample_rate, n_mfcc, n_fft, hop_length)
    return torch.cat([f(waves[s:s + chunk]) for s in range(0, waves.shape[0], chunk)])


class SmallCNN(nn.Module):
    """utils/models.py:17-65 restated (same submodule names -> same state_dict keys)."""

    def __init__(self, num_classes: int, linear_features: int):
        super().__init__()
        self.conv1 = nn.Conv2d(1, 64, (2, 2))
        self.bn1 = nn.BatchNorm2d(64)
        self.conv2 = nn.Conv2d(64, 64, (2, 2))
        self.bn2 = nn.BatchNorm2d(64)
        self.conv3 = nn.Conv2d(64, 32, (2, 2))
        self.bn3 = nn.BatchNorm2d(32)
        self.fc1 = nn.Linear(linear_features, 128)
        self.fc2 = nn.Linear(128, num_classes)

    def forward(self, x):
        x = Fn.max_pool2d(self.bn1(Fn.relu(self.conv1(x))), (1, 3))
        x = Fn.max_pool2d(self.bn2(Fn.relu(self.conv2(x))), (2, 2), padding=(1, 1))
        x = Fn.max_pool2d(self.bn3(Fn.relu(self.conv3(x))), (2, 2), padding=(0, 1))
        x = Fn.dropout(x, 0.4, self.training).flatten(1)
        x = Fn.dropout(Fn.relu(self.fc1(x)), 0.5, self.training)
        return Fn.log_softmax(self.fc2(x), dim=1)


def train_step(model, opt, x, y, ind):
    """One iteration of utils/training_tools.py:60-79; returns (loss, correct, poison_total, asr_correct)."""
    opt.zero_grad()
    out = model(x)
    loss = Fn.cross_entropy(out, y)
    loss.backward()
    opt.step()
    pred = out.max(1)[1]
    hit = pred.eq(y)
    p = ind == 1
    return float(loss.item()), int(hit.sum()), int(p.sum()), int((hit & p).sum())
