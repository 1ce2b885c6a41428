"""PyTorch custom ops over libabd: the ``abd`` operator namespace (north_star
"surfaced as PyTorch-ROCm custom ops").

    torch.ops.abd.mfcc                 prepare_dataset.py:35-47 (+ the fused trigger injection)
    torch.ops.abd.inject_waveform      ultrasonic.py:75, flowmur.py:77-85 / 101-106
    torch.ops.abd.smallcnn_eval        utils/models.py:43-65 in eval mode
    torch.ops.abd.smallcnn_eval_metrics  the same + test()'s counters (utils/training_tools.py:98-128)
    torch.ops.abd.smallcnn_train_step  utils/training_tools.py:60-79: forward, CE, backward, Adam,
                                       loss / accuracy / ASR counters -- one launch sequence
    torch.ops.abd.adam                 torch.optim.Adam single-tensor step (flat buffers)

Each op enqueues its HIP kernels on the current torch stream through the C ABI
(include/abd.h) and has a fake (meta) implementation, so the ops trace under FakeTensor /
torch.compile-style tooling and pass ``torch.library.opcheck`` (tests/test_gpu_ops.py).  The
mutating ops declare what they write (params, grads, Adam moments, BN buffers, counters).
There is no CPU kernel: a CPU tensor raises AbdError (no silent fallback).

The drop-in shims route through these ops (features.MFCC, training.train / test, the
smallcnn eval forward); the HBM-resident bench loop (pipeline.ResidentTrainer) calls the same C
entry points directly to skip the Python dispatcher (~2 x 20 us per step).
"""
from __future__ import annotations

import ctypes as C
from typing import Optional

import torch
from torch import Tensor

from . import _lib as L
from . import features as F

_NETS: dict = {}


def n_frames(length, n_fft: int, hop: int):
    """center=True frame count (torch.stft / librosa): 1 + (L + 2 (n_fft // 2) - n_fft) // hop."""
    return 1 + (length + 2 * (n_fft // 2) - n_fft) // hop


def _net(H0: int, W0: int, K: int, precision: str = "f32split"):
    """A cached libabd network handle for one geometry (no device state: shapes and precision)."""
    key = (int(H0), int(W0), int(K))
    h = _NETS.get(key)
    if h is None:
        h = C.c_void_p()
        L.check(L.lib().abd_smallcnn_create(key[0], key[1], key[2], 0, C.byref(h)), "abd_smallcnn_create")
        _NETS[key] = h
    L.check(L.lib().abd_smallcnn_set_precision(h, L.PRECISIONS[precision]), "abd_smallcnn_set_precision")
    return h


def _ws(n_bytes: int, device) -> Tensor:
    return torch.empty(max(int(n_bytes), 1), dtype=torch.uint8, device=device)


def _ptr(t: Optional[Tensor]):
    return t.data_ptr() if t is not None else None


# --------------------------------------------------------------------------- features
@torch.library.custom_op("abd::mfcc", mutates_args=())
def mfcc(waves: Tensor, sample_rate: int, n_mfcc: int, n_fft: int, hop_length: int, mel: str = "htk",
         pad: str = "reflect", rows: Optional[Tensor] = None, inject_mode: int = 0,
         trigger: Optional[Tensor] = None, poison: Optional[Tensor] = None, position: Optional[Tensor] = None,
         snr_db: float = 30.0, patch_box: Optional[list[int]] = None, patch_value: float = -200.0) -> Tensor:
    """(N, L) fp32 waves -> (B, 1, T, n_mfcc): torchaudio T.MFCC (mel 'htk', pad 'reflect') or librosa
    (mel 'slaney', pad 'constant'), with optional trigger injection fused into the load / epilogue."""
    L.require_device(waves, "waves")
    cfg = F.MfccConfig(int(sample_rate), int(n_mfcc), int(n_fft), int(hop_length), int(waves.shape[1]), mel=mel,
                       pad=pad)
    inj = None
    if inject_mode or patch_box is not None:
        inj = F.Injection(mode=int(inject_mode), trigger=trigger, poison=poison, position=position,
                          snr_db=float(snr_db),
                          patch=(tuple(patch_box) + (float(patch_value),)) if patch_box is not None else None)
    return F.mfcc_batch(waves, cfg, rows=rows, inject=inj)


@mfcc.register_fake
def _(waves, sample_rate, n_mfcc, n_fft, hop_length, mel="htk", pad="reflect", rows=None, inject_mode=0,
      trigger=None, poison=None, position=None, snr_db=30.0, patch_box=None, patch_value=-200.0):
    B = rows.shape[0] if rows is not None else waves.shape[0]
    return waves.new_empty((B, 1, n_frames(waves.shape[1], n_fft, hop_length), n_mfcc))


@torch.library.custom_op("abd::inject_waveform", mutates_args=())
def inject_waveform(waves: Tensor, trigger: Tensor, mode: int, poison: Optional[Tensor] = None,
                    position: Optional[Tensor] = None, snr_db: float = 30.0) -> Tensor:
    """The poisoned waveforms (N, L) themselves (the reference's bd_*_wav arrays)."""
    inj = F.Injection(mode=int(mode), trigger=trigger, poison=poison, position=position, snr_db=float(snr_db))
    return F.inject_waveform(waves, int(waves.shape[1]), inj)


@inject_waveform.register_fake
def _(waves, trigger, mode, poison=None, position=None, snr_db=30.0):
    return torch.empty_like(waves)


# --------------------------------------------------------------------------- smallcnn
def _eval(x, params, running, num_classes, precision, labels, indicators, metrics):
    L.require_device(x, "smallcnn input")
    B, H0, W0 = int(x.shape[0]), int(x.shape[2]), int(x.shape[3])
    h = _net(H0, W0, num_classes, precision)
    out = torch.empty((B, int(num_classes)), dtype=torch.float32, device=x.device)
    ws = _ws(L.lib().abd_smallcnn_workspace_bytes(h, B), x.device)
    L.check(L.lib().abd_smallcnn_eval(h, x.data_ptr(), B, params.data_ptr(), running.data_ptr(), _ptr(labels),
                                      _ptr(indicators), out.data_ptr(), _ptr(metrics), ws.data_ptr(), ws.numel(),
                                      L.stream_ptr(x.device)), "abd_smallcnn_eval")
    return out


@torch.library.custom_op("abd::smallcnn_eval", mutates_args=())
def smallcnn_eval(x: Tensor, params: Tensor, running: Tensor, num_classes: int, precision: str = "f32split") -> Tensor:
    """model.eval() forward: (B, 1, H0, W0) -> log-probs (B, K); running BN statistics, no dropout."""
    return _eval(x, params, running, num_classes, precision, None, None, None)


@smallcnn_eval.register_fake
def _(x, params, running, num_classes, precision="f32split"):
    return x.new_empty((x.shape[0], num_classes))


@torch.library.custom_op("abd::smallcnn_eval_metrics", mutates_args=("metrics",))
def smallcnn_eval_metrics(x: Tensor, params: Tensor, running: Tensor, num_classes: int, precision: str,
                          labels: Tensor, indicators: Optional[Tensor], metrics: Tensor) -> Tensor:
    """The eval forward plus test()'s loss / accuracy / ASR counters accumulated into metrics
    (int64[8]; utils/training_tools.py:98-128); returns the log-probs."""
    return _eval(x, params, running, num_classes, precision, labels, indicators, metrics)


@smallcnn_eval_metrics.register_fake
def _(x, params, running, num_classes, precision, labels, indicators, metrics):
    return x.new_empty((x.shape[0], num_classes))


@torch.library.custom_op("abd::smallcnn_train_step",
                         mutates_args=("params", "grads", "exp_avg", "exp_avg_sq", "running", "num_batches_tracked",
                                       "metrics"))
def smallcnn_train_step(x: Tensor, labels: Tensor, indicators: Optional[Tensor], params: Tensor, grads: Tensor,
                        exp_avg: Tensor, exp_avg_sq: Tensor, running: Tensor, num_batches_tracked: Tensor,
                        metrics: Tensor, num_classes: int, adam_step: int, lr: float, beta1: float, beta2: float,
                        eps: float, seed: int, counter: int, mask1: Optional[Tensor] = None,
                        mask2: Optional[Tensor] = None, precision: str = "f32split", grad_scale: float = 1.0,
                        row_offset: int = 0) -> Tensor:
    """One fused train() iteration on the device; returns the batch's log-probs (B, K).

    adam_step >= 1 applies torch.optim.Adam (that step index); 0 leaves params untouched (data
    parallelism: grads are all-reduced first, then abd::adam).  metrics (int64[8]) accumulates
    loss / samples / correct / poisoned / ASR hits / batches like train()."""
    L.require_device(x, "smallcnn input")
    B, H0, W0 = int(x.shape[0]), int(x.shape[2]), int(x.shape[3])
    h = _net(H0, W0, num_classes, precision)
    out = torch.empty((B, int(num_classes)), dtype=torch.float32, device=x.device)
    a = L.TrainArgs()
    a.x, a.batch = x.data_ptr(), B
    a.labels, a.indicators = labels.data_ptr(), _ptr(indicators)
    a.params, a.grads, a.running = params.data_ptr(), grads.data_ptr(), running.data_ptr()
    a.exp_avg, a.exp_avg_sq = exp_avg.data_ptr(), exp_avg_sq.data_ptr()
    a.num_batches_tracked = num_batches_tracked.data_ptr()
    a.lr, a.beta1, a.beta2, a.eps = float(lr), float(beta1), float(beta2), float(eps)
    a.adam_step, a.do_update = int(adam_step), 1 if adam_step > 0 else 0
    a.seed, a.counter, a.row_offset = int(seed), int(counter), int(row_offset)
    a.mask1_in, a.mask2_in = _ptr(mask1), _ptr(mask2)
    a.logprobs_out, a.metrics, a.grad_scale = out.data_ptr(), metrics.data_ptr(), float(grad_scale)
    ws = _ws(L.lib().abd_smallcnn_workspace_bytes(h, B), x.device)
    L.check(L.lib().abd_smallcnn_train_step(h, C.byref(a), ws.data_ptr(), ws.numel(), L.stream_ptr(x.device)),
            "abd_smallcnn_train_step")
    return out


@smallcnn_train_step.register_fake
def _(x, labels, indicators, params, grads, exp_avg, exp_avg_sq, running, num_batches_tracked, metrics, num_classes,
      adam_step, lr, beta1, beta2, eps, seed, counter, mask1=None, mask2=None, precision="f32split", grad_scale=1.0,
      row_offset=0):
    return x.new_empty((x.shape[0], num_classes))


@torch.library.custom_op("abd::adam", mutates_args=("params", "exp_avg", "exp_avg_sq"))
def adam(params: Tensor, grads: Tensor, exp_avg: Tensor, exp_avg_sq: Tensor, step: int, lr: float, beta1: float,
         beta2: float, eps: float) -> None:
    """torch.optim.Adam single-tensor update over flat fp32 buffers (weight_decay 0)."""
    L.require_device(params, "params")
    L.check(L.lib().abd_adam_f32(params.data_ptr(), grads.data_ptr(), exp_avg.data_ptr(), exp_avg_sq.data_ptr(),
                                 params.numel(), int(step), float(lr), float(beta1), float(beta2), float(eps),
                                 L.stream_ptr(params.device)), "abd_adam_f32")


@adam.register_fake
def _(params, grads, exp_avg, exp_avg_sq, step, lr, beta1, beta2, eps):
    return None
