"""Feature stage host API: fused trigger injection + MFCC on the HIP device.

Mirrors the reference's feature entry points:
  * ``MFCC(waveform, sample_rate, n_mfcc, n_fft, hop_length)``  -- prepare_dataset.py:35-47
    (torchaudio T.MFCC; (L,) -> (n_mfcc, T), (N,1,L) -> (N,1,n_mfcc,T))
  * ``librosa_MFCC(waveform, sample_rate, n_mfcc)``           -- utils/daba_selection_tools.py:16-22
and exposes the batched GPU form the training pipeline uses:
  * ``mfcc_batch(waves, ..., rows=, inject=)`` -> (B, 1, T, n_mfcc), the model input
    layout (``MFCC(..).numpy().T[np.newaxis]`` stacked, prepare_dataset.py:65).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np
import torch

from . import _lib as L


@dataclass(frozen=True)
class MfccConfig:
    sample_rate: int
    n_mfcc: int
    n_fft: int
    hop_length: int
    length: int
    mel: str = "htk"          # 'htk' (torchaudio) | 'slaney' (librosa)
    pad: str = "reflect"      # 'reflect' (torchaudio) | 'constant' (librosa >= 0.10)
    n_mels: int = 128
    top_db: float = 80.0

    @staticmethod
    def torchaudio(sample_rate, n_mfcc, n_fft, hop_length, length):
        return MfccConfig(int(sample_rate), int(n_mfcc), int(n_fft), int(hop_length), int(length))

    @staticmethod
    def librosa(sample_rate, n_mfcc, length, n_fft=2048, hop_length=512, pad="constant"):
        return MfccConfig(int(sample_rate), int(n_mfcc), int(n_fft), int(hop_length), int(length),
                          mel="slaney", pad=pad)


class MfccPlan:
    """Device tables (twiddles, Bluestein chirps, sparse mel filterbank, DCT) for one config."""

    def __init__(self, cfg: MfccConfig, device=None):
        self.cfg = cfg
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        lib = L.lib()
        h = C.c_void_p()
        with torch.cuda.device(self.device):
            rc = lib.abd_mfcc_plan_create(cfg.sample_rate, cfg.n_fft, cfg.hop_length, cfg.n_mels, cfg.n_mfcc,
                                          L.ABD_MEL_HTK if cfg.mel == "htk" else L.ABD_MEL_SLANEY,
                                          L.ABD_PAD_REFLECT if cfg.pad == "reflect" else L.ABD_PAD_CONSTANT,
                                          float(cfg.top_db), cfg.length, C.byref(h))
        L.check(rc, "abd_mfcc_plan_create")
        self._h = h
        self.n_frames = lib.abd_mfcc_plan_frames(h)

    def describe(self):
        m, blue, npass = C.c_int(), C.c_int(), C.c_int()
        rad = (C.c_int * 16)()
        L.check(L.lib().abd_mfcc_plan_describe(self._h, C.byref(m), C.byref(blue), C.byref(npass), rad), "describe")
        return {"fft_size": m.value, "bluestein": bool(blue.value), "radices": list(rad[:npass.value]),
                "n_frames": self.n_frames}

    def workspace_bytes(self, batch: int) -> int:
        return int(L.lib().abd_mfcc_workspace_bytes(self._h, int(batch)))

    def workspace(self, batch: int) -> torch.Tensor:
        """A fresh workspace for one launch of ``batch`` rows, from the caching allocator on the
        current stream.  The plan itself holds no per-call device state (ops are
        re-entrant): two launches on two streams get two workspaces, so neither the STFT's item
        queues (zeroed per launch) nor its dB intermediate can be shared between them."""
        return torch.empty(max(self.workspace_bytes(batch), 1), dtype=torch.uint8, device=self.device)

    def __del__(self):
        try:
            if getattr(self, "_h", None) and self._h.value:
                L.lib().abd_mfcc_plan_destroy(self._h)
        except Exception:
            pass


_PLANS: dict = {}


def get_plan(cfg: MfccConfig, device=None) -> MfccPlan:
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    key = (cfg, dev.index)
    p = _PLANS.get(key)
    if p is None:
        p = MfccPlan(cfg, dev)
        _PLANS[key] = p
    return p


@dataclass
class Injection:
    """Trigger injection fused into the feature kernel (see include/abd.h abd_inject)."""
    mode: int = L.INJECT_NONE
    trigger: torch.Tensor | None = None      # float32 (Lt,) on device
    poison: torch.Tensor | None = None       # uint8 (B,) on device; None = every row
    position: torch.Tensor | None = None     # int32 (B,) on device (windowed modes)
    snr_db: float = 30.0
    patch: tuple | None = None               # (t0, t1, c0, c1, value): BadNets MFCC patch
    frames: torch.Tensor | None = None       # int32 (B,) valid frames per row (ragged clips), None = all
    frame_pad: float = -200.0                # value of the frames past a ragged row's end
    row_scale: torch.Tensor | None = None    # float32 (N,) per TABLE row (row_scales()), None = per call

    def to_c(self) -> L.Inject:
        s = L.Inject()
        s.mode = int(self.mode)
        if self.trigger is not None:
            L.require_device(self.trigger, "trigger")
            assert self.trigger.dtype == torch.float32
            s.trigger = self.trigger.data_ptr()
            s.trigger_len = self.trigger.numel()
        if self.poison is not None:
            assert self.poison.dtype == torch.uint8
            s.poison = self.poison.data_ptr()
        if self.position is not None:
            assert self.position.dtype == torch.int32
            s.position = self.position.data_ptr()
        s.snr_db = float(self.snr_db)
        if self.patch is not None:
            s.patch = 1
            s.patch_t0, s.patch_t1, s.patch_c0, s.patch_c1 = (int(v) for v in self.patch[:4])
            s.patch_value = float(self.patch[4])
        if self.frames is not None:
            assert self.frames.dtype == torch.int32 and self.frames.is_cuda
            s.frames = self.frames.data_ptr()
            s.frame_pad = float(self.frame_pad)
        if self.row_scale is not None:
            assert self.row_scale.dtype == torch.float32 and self.row_scale.is_cuda
            s.row_scale = self.row_scale.data_ptr()
        return s


def mfcc_batch(waves: torch.Tensor, cfg: MfccConfig, rows: torch.Tensor | None = None,
               inject: Injection | None = None, out: torch.Tensor | None = None,
               batch: int | None = None, workspace: torch.Tensor | None = None) -> torch.Tensor:
    """waves (N, >=L) fp32 on device -> (B, 1, T, n_mfcc); rows (int32, B) gathers the batch.

    ``workspace`` (uint8, >= ``plan.workspace_bytes(B)``) is caller-owned scratch; the caller
    orders its reuse (the resident trainer keeps one per stream).  Without it each call takes a
    fresh block from the caching allocator on the current stream, so concurrent calls on
    different streams never share scratch."""
    L.require_device(waves, "waves")
    assert waves.dtype == torch.float32 and waves.dim() == 2 and waves.shape[1] >= cfg.length
    plan = get_plan(cfg, waves.device)
    if rows is not None:
        assert rows.dtype == torch.int32 and rows.is_cuda
        B = rows.numel() if batch is None else batch
    else:
        B = waves.shape[0] if batch is None else batch
    if out is None:
        out = torch.empty((B, 1, plan.n_frames, cfg.n_mfcc), dtype=torch.float32, device=waves.device)
    if workspace is None:
        ws = plan.workspace(B)
    else:
        assert workspace.dtype == torch.uint8 and workspace.is_cuda and workspace.numel() >= plan.workspace_bytes(B)
        ws = workspace
    inj = inject.to_c() if inject is not None else None
    rc = L.lib().abd_mfcc_f32(plan._h, waves.data_ptr(), waves.stride(0),
                             rows.data_ptr() if rows is not None else None, B,
                             C.byref(inj) if inj is not None else None, out.data_ptr(),
                             ws.data_ptr(), ws.numel(), L.stream_ptr(waves.device))
    L.check(rc, "abd_mfcc_f32")
    return out


def row_scales(waves: torch.Tensor, length: int, inject: Injection) -> torch.Tensor:
    """The SNR_WINDOW / DEPLOY mixing scale of every row of a resident wave table (flowmur.py:77-80,
    flowmur_generate_trigger.py:50-52), for ``Injection.row_scale``: the reference mixes each clip
    once, offline, so a table whose rows and trigger stay fixed needs its scales only once."""
    L.require_device(waves, "waves")
    out = torch.empty(waves.shape[0], dtype=torch.float32, device=waves.device)
    inj = inject.to_c()
    rc = L.lib().abd_inject_row_scales(waves.data_ptr(), waves.stride(0), length, waves.shape[0], C.byref(inj),
                                      out.data_ptr(), L.stream_ptr(waves.device))
    L.check(rc, "abd_inject_row_scales")
    return out


def inject_waveform(waves: torch.Tensor, length: int, inject: Injection, rows: torch.Tensor | None = None):
    """The poisoned waveform itself (B, L) -- the reference's bd_*_wav arrays."""
    L.require_device(waves, "waves")
    B = rows.numel() if rows is not None else waves.shape[0]
    out = torch.empty((B, length), dtype=torch.float32, device=waves.device)
    need = L.lib().abd_inject_workspace_bytes(B)
    ws = torch.empty(max(need, 1), dtype=torch.uint8, device=waves.device)
    inj = inject.to_c()
    rc = L.lib().abd_inject_waveform_f32(waves.data_ptr(), waves.stride(0), length,
                                        rows.data_ptr() if rows is not None else None, B, C.byref(inj),
                                        out.data_ptr(), ws.data_ptr(), ws.numel(), L.stream_ptr(waves.device))
    L.check(rc, "abd_inject_waveform_f32")
    return out


def _device():
    if not torch.cuda.is_available():
        raise L.AbdError("no ROCm/HIP device visible: the abd MFCC runs on MI355X only (no CPU fallback)")
    return torch.device("cuda", torch.cuda.current_device())


def MFCC(waveform, sample_rate, n_mfcc, n_fft, hop_length):
    """Drop-in for prepare_dataset.MFCC (prepare_dataset.py:35-47), computed on the HIP device.

    (L,) -> (n_mfcc, T); (N,1,L) -> (N,1,n_mfcc,T); result on the input's device.
    """
    t = waveform if isinstance(waveform, torch.Tensor) else torch.as_tensor(np.asarray(waveform))
    src_dev = t.device
    dev = t.device if t.is_cuda else _device()
    x = t.to(device=dev, dtype=torch.float32)
    from . import ops  # noqa: F401  (registers torch.ops.abd)
    if x.dim() == 1:
        y = torch.ops.abd.mfcc(x.reshape(1, -1).contiguous(), int(sample_rate), int(n_mfcc), int(n_fft),
                               int(hop_length))[0, 0].transpose(0, 1)
    elif x.dim() == 3 and x.shape[1] == 1:
        y = torch.ops.abd.mfcc(x[:, 0].contiguous(), int(sample_rate), int(n_mfcc), int(n_fft),
                               int(hop_length)).transpose(2, 3)
    else:
        raise ValueError("MFCC supports (L,) and (N,1,L) waveforms (the reference's call shapes)")
    return y.contiguous().to(src_dev)


def librosa_MFCC(waveform, sample_rate, n_mfcc):
    """Drop-in for librosa_MFCC (utils/daba_selection_tools.py:16-22): (L,) float -> (n_mfcc, T) float64."""
    x = torch.as_tensor(np.asarray(waveform, dtype=np.float32), device=_device()).reshape(1, -1).contiguous()
    cfg = MfccConfig.librosa(sample_rate, n_mfcc, x.shape[1])
    y = mfcc_batch(x, cfg)[0, 0].transpose(0, 1)
    return y.cpu().numpy().astype(np.float64)


class ResamplePlan:
    """Device polyphase sinc table for one (orig, new) rate pair (libabd abd_resample_*)."""

    def __init__(self, orig_freq, new_freq, lowpass_filter_width=6, rolloff=0.99):
        h = C.c_void_p()
        L.check(L.lib().abd_resample_plan_create(int(orig_freq), int(new_freq), int(lowpass_filter_width),
                                                 float(rolloff), C.byref(h)), "abd_resample_plan_create")
        self._h = h

    def output_length(self, length):
        return int(L.lib().abd_resample_output_length(self._h, int(length)))

    def __del__(self):
        try:
            if getattr(self, "_h", None) and self._h.value:
                L.lib().abd_resample_plan_destroy(self._h)
        except Exception:
            pass


_RS_PLANS: dict = {}


def resample(waveform, orig_freq, new_freq, lowpass_filter_width=6, rolloff=0.99):
    """torchaudio.functional.resample (sinc_interp_hann) on the HIP device -- prepare_dataset.py:60.

    (..., L) float -> (..., ceil(new * L / orig)) on the input's device; equal rates return the input."""
    t = waveform if isinstance(waveform, torch.Tensor) else torch.as_tensor(np.asarray(waveform))
    if int(orig_freq) == int(new_freq):
        return t
    src_dev = t.device
    dev = t.device if t.is_cuda else _device()
    shape = t.shape
    x = t.to(device=dev, dtype=torch.float32).reshape(-1, shape[-1]).contiguous()
    key = (int(orig_freq), int(new_freq), int(lowpass_filter_width), float(rolloff), dev.index)
    plan = _RS_PLANS.get(key)
    if plan is None:
        with torch.cuda.device(dev):
            plan = ResamplePlan(orig_freq, new_freq, lowpass_filter_width, rolloff)
        _RS_PLANS[key] = plan
    n_out = plan.output_length(x.shape[1])
    out = torch.empty((x.shape[0], n_out), dtype=torch.float32, device=dev)
    L.check(L.lib().abd_resample_f32(plan._h, x.data_ptr(), x.stride(0), x.shape[0], x.shape[1], out.data_ptr(),
                                     out.stride(0), L.stream_ptr(dev)), "abd_resample_f32")
    return out.reshape(tuple(shape[:-1]) + (n_out,)).to(src_dev)
