"""Synthetic class-conditional 1 s clips: the dataset is not in the image.

Class c: two sinusoids at class-specific frequencies with random phase, a 3-8 Hz
amplitude envelope and N(0, 0.05^2) noise, clipped to [-1, 1] and quantised to
int16/32768 like torchaudio.load (prepare_dataset.py:59, pinned by test.ipynb cell 12).
"""
from __future__ import annotations

import math

import numpy as np
import torch


def class_freqs(c: int, sr: int):
    nyq = sr / 2.0
    f1 = 180.0 + 97.0 * c
    f2 = 900.0 + 331.0 * c
    return min(f1, 0.45 * nyq), min(f2, 0.45 * nyq)


def make_clips_np(n, sr, length, num_classes, seed=35):
    """numpy PCG64 version (small n; tests)."""
    r = np.random.Generator(np.random.PCG64(seed))
    labels = r.integers(0, num_classes, n).astype(np.int64)
    t = np.arange(length) / sr
    out = np.empty((n, length), dtype=np.float32)
    for i in range(n):
        f1, f2 = class_freqs(int(labels[i]), sr)
        ph = r.uniform(0, 2 * math.pi, 3)
        env = 0.6 + 0.4 * np.sin(2 * math.pi * r.uniform(3, 8) * t + ph[2])
        x = env * (0.35 * np.sin(2 * math.pi * f1 * t + ph[0]) + 0.2 * np.sin(2 * math.pi * f2 * t + ph[1]))
        x = x + r.normal(0.0, 0.05, length)
        q = np.clip(np.round(np.clip(x, -1.0, 1.0) * 32768.0), -32768, 32767)
        out[i] = (q / 32768.0).astype(np.float32)
    return out, labels


def make_clips_torch(n, sr, length, num_classes, seed=35, device="cuda", chunk=2048):
    """Same distribution generated on the device (bench-scale data, not bit-identical to the numpy one)."""
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    labels = torch.randint(0, num_classes, (n,), generator=g, device=device)
    waves = torch.empty((n, length), dtype=torch.float32, device=device)
    t = torch.arange(length, device=device, dtype=torch.float32) / sr
    f1 = torch.tensor([class_freqs(c, sr)[0] for c in range(num_classes)], device=device)
    f2 = torch.tensor([class_freqs(c, sr)[1] for c in range(num_classes)], device=device)
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        lab = labels[s:e]
        ph = torch.rand((e - s, 3), generator=g, device=device) * (2 * math.pi)
        am = 3.0 + 5.0 * torch.rand((e - s, 1), generator=g, device=device)
        env = 0.6 + 0.4 * torch.sin(2 * math.pi * am * t + ph[:, 2:3])
        x = env * (0.35 * torch.sin(2 * math.pi * f1[lab, None] * t + ph[:, 0:1])
                   + 0.2 * torch.sin(2 * math.pi * f2[lab, None] * t + ph[:, 1:2]))
        x = x + 0.05 * torch.randn((e - s, length), generator=g, device=device)
        waves[s:e] = torch.clamp(torch.round(torch.clamp(x, -1.0, 1.0) * 32768.0), -32768, 32767) / 32768.0
    return waves, labels
