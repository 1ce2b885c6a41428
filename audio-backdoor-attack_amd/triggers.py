"""Trigger APIs with the reference's signatures (host side of the injection kernels).

* BadNets  ``generate_trigger`` / ``add_trigger_to_mfcc``       utils/badnet_trigger.py:4-27
* Ultrasonic ``GenerateTrigger`` / ``TriggerInfeasible``        utils/ultra_trigger.py:8-111
* FlowMur  ``deploy_trigger_to_waveform``                       utils/flowmur_generate_trigger.py:49-62
* DABA     ``single_trigger_injection_db`` on int16 arrays      utils/daba_selection_tools.py:24-39
* JingleBack ``get_boards`` / ``poison_style``                  utils/styles_trigger.py:8-53 (libabd effects kernels + pitch stage)

Trigger *construction* is a one-off host computation (microseconds, once per run);
trigger *application* per batch happens inside libabd's feature kernel
(features.Injection).  The standalone application helpers below also run on the
device through libabd.
"""
from __future__ import annotations

import ctypes as C
import math
import os

import numpy as np
import torch

from . import _lib as L

_RES = os.path.join(os.path.dirname(os.path.abspath(__file__)), "resources")


# ------------------------------------------------------------------ BadNets
def generate_trigger(image_width, image_height, square_size, distance_to_right=0, distance_to_bottom=0, save=True):
    """(1, H, W) float64 zeros with a -200 square at the bottom-right (last frames x last coefficients)."""
    trig = np.zeros((1, image_height, image_width))
    r1 = image_height - distance_to_bottom
    c1 = image_width - distance_to_right
    trig[:, r1 - square_size:r1, c1 - square_size:c1] = -200
    if save:
        os.makedirs("resources/BadNets", exist_ok=True)
        np.save("resources/BadNets/trigger.npy", trig)
    return trig


def add_trigger_to_mfcc(mfcc, trigger_matrix):
    """In-place overwrite of mfcc at the trigger's non-zero cells (returns the same array)."""
    sel = trigger_matrix != 0
    mfcc[sel] = trigger_matrix[sel]
    return mfcc


def patch_spec(trigger_matrix) -> tuple:
    """Bounding rectangle + value of a BadNets trigger, for the fused MFCC epilogue."""
    nz = np.argwhere(np.asarray(trigger_matrix)[0] != 0)
    if nz.size == 0:
        return None
    (t0, c0), (t1, c1) = nz.min(axis=0), nz.max(axis=0) + 1
    vals = np.asarray(trigger_matrix)[0, t0:t1, c0:c1]
    if not np.all(vals == vals.flat[0]):
        raise ValueError("fused patch epilogue expects a constant rectangular trigger")
    return (int(t0), int(t1), int(c0), int(c1), float(vals.flat[0]))


# ------------------------------------------------------------------ Ultrasonic
class TriggerInfeasible(Exception):
    """Bad (size, pos) for the ultrasonic trigger (utils/ultra_trigger.py:8-24)."""

    correct_pos = ["start", "mid", "end"]
    correct_size = 60

    def __init__(self, size, pos):
        self.size, self.pos = size, pos
        self.message = (f"Cannot apply trigger (size: {size}, pos: {pos}). Size should be in (0, "
                        f"{self.correct_size}] and pos should be in {self.correct_pos}")
        super().__init__(self.message)


class GenerateTrigger:
    """Gated 44.1 kHz ultrasonic tone; samples ship as resources/ultrasonic_trigger_int16.npy
    (the reference's resources/Ultrasonic/trigger.wav data, normalised /32768 like torchaudio.load)."""

    divider = 100

    def __init__(self, size, pos, cont=True, debug=False):
        if pos not in ("start", "mid", "end") or size <= 0 or size > self.divider:
            raise TriggerInfeasible(size, pos)
        self.data = (np.load(os.path.join(_RES, "ultrasonic_trigger_int16.npy")).astype(np.float32) / 32768.0)[None]
        self.sample_rate = 44100
        self.points = (self.data.shape[1] // self.divider) * size
        self.size, self.pos, self.cont, self.debug = size, pos, cont, debug

    def _keep_mask(self):
        L_ = self.data.shape[1]
        keep = np.zeros(L_, dtype=bool)
        if self.cont:
            if self.pos == "start":
                lo, hi = 0, self.points - 1
            elif self.pos == "mid":
                lo = L_ // 2 - self.points // 2 + (self.points % 2)
                hi = L_ // 2 + self.points // 2 - 1
            else:
                lo, hi = L_ - self.points, L_ - 1
            keep[lo:hi + 1] = True
        else:
            seg = int(self.points / 5)
            for k in range(5):
                keep[k * (L_ // 5):k * (L_ // 5) + seg] = True
        return keep

    def trigger(self):
        self.data[:, ~self._keep_mask()] = 0
        return self.data


# ------------------------------------------------------------------ FlowMur
def deploy_trigger_to_waveform(waveforms, trigger, positions=None, seed=None):
    """(B,1,L) waves, (1,Lt) trigger -> (B,1,L) mixed at SNR 30 dB on the HIP device.

    The reference draws each position with python ``random.randint`` (inclusive);
    pass ``positions`` to pin them."""
    from . import features as F
    w = torch.as_tensor(waveforms)
    dev = w.device if w.is_cuda else torch.device("cuda", torch.cuda.current_device())
    wd = w.to(dev, torch.float32).reshape(w.shape[0], -1).contiguous()
    t = torch.as_tensor(trigger).to(dev, torch.float32).reshape(-1).contiguous()
    if positions is None:
        import random
        rnd = random.Random(seed) if seed is not None else random
        positions = [rnd.randint(0, wd.shape[1] - t.numel()) for _ in range(wd.shape[0])]
    pos = torch.as_tensor(np.asarray(positions, dtype=np.int32), device=dev)
    out = F.inject_waveform(wd, wd.shape[1], F.Injection(mode=L.INJECT_DEPLOY, trigger=t, position=pos))
    return out.reshape(w.shape[0], 1, -1).to(w.device)


# ------------------------------------------------------------------ DABA (pydub int16 semantics)
def dbfs_int16(x: np.ndarray) -> float:
    """AudioSegment.dBFS: 20 log10(int(rms) / 32768) (audioop.rms truncates)."""
    x = np.asarray(x, dtype=np.float64)
    r = int(math.sqrt(float(np.dot(x, x)) / x.size)) if x.size else 0
    return -math.inf if r == 0 else 20.0 * math.log10(r / 32768.0)


def db_to_float(db: float) -> float:
    """pydub.utils.db_to_float: the linear factor AudioSegment + dB hands audioop.mul."""
    return 10 ** (float(db) / 20)


def single_trigger_injection_db(host_int16, trig_int16, po_db):
    """song1.overlay(song2 + (po_db - song2.dBFS)) on int16 samples, computed by libabd."""
    h = np.asarray(host_int16, dtype=np.int16)
    t = np.asarray(trig_int16, dtype=np.int16)
    if po_db == "keep":
        gain = 0.0
    elif po_db == "auto":
        gain = dbfs_int16(h) - dbfs_int16(t)
    else:
        gain = float(po_db) - dbfs_int16(t)
    dev = torch.device("cuda", torch.cuda.current_device())
    hd = torch.tensor(h[None], device=dev)
    td = torch.tensor(t[None], device=dev)
    gd = torch.tensor([db_to_float(gain)], dtype=torch.float64, device=dev)
    out = torch.empty_like(hd)
    L.check(L.lib().abd_pydub_overlay_i16(hd.data_ptr(), h.size, td.data_ptr(), t.size, gd.data_ptr(), 1,
                                          out.data_ptr(), L.stream_ptr(dev)), "abd_pydub_overlay_i16")
    return out[0].cpu().numpy()


# ------------------------------------------------------------------ JingleBack (pedalboard)
class _Effect:
    """A pedalboard plugin description (utils/styles_trigger.py:5); run by libabd's style board."""
    kind = None

    def params(self):
        return []

    def __repr__(self):
        return f"{type(self).__name__}({', '.join(f'{v:g}' for v in self.params())})"


class Gain(_Effect):
    kind = L.FX_GAIN

    def __init__(self, gain_db=1.0):
        self.gain_db = float(gain_db)

    def params(self):
        return [self.gain_db]


class Distortion(_Effect):
    kind = L.FX_DISTORTION

    def __init__(self, drive_db=25.0):
        self.drive_db = float(drive_db)

    def params(self):
        return [self.drive_db]


class LadderFilter(_Effect):
    kind = L.FX_LADDER

    class Mode:
        LPF12, HPF12, BPF12, LPF24, HPF24, BPF24 = 0, 1, 2, 3, 4, 5

    def __init__(self, mode=0, cutoff_hz=200.0, resonance=0.0, drive=1.0):
        self.mode, self.cutoff_hz, self.resonance, self.drive = int(mode), float(cutoff_hz), float(resonance), \
            float(drive)

    def params(self):
        return [self.mode, self.cutoff_hz, self.resonance, self.drive]


class Phaser(_Effect):
    kind = L.FX_PHASER

    def __init__(self, rate_hz=1.0, depth=0.5, centre_frequency_hz=1300.0, feedback=0.0, mix=0.5):
        self.rate_hz, self.depth, self.centre_frequency_hz = float(rate_hz), float(depth), float(centre_frequency_hz)
        self.feedback, self.mix = float(feedback), float(mix)

    def params(self):
        return [self.rate_hz, self.depth, self.centre_frequency_hz, self.feedback, self.mix]


class Chorus(_Effect):
    """pedalboard.Chorus (juce::dsp::Chorus); feedback must be 0, and only Gain / Distortion (after
    an opening PitchShift) may precede it in a board."""
    kind = L.FX_CHORUS

    def __init__(self, rate_hz=1.0, depth=0.25, centre_delay_ms=7.0, feedback=0.0, mix=0.5):
        self.rate_hz, self.depth, self.centre_delay_ms = float(rate_hz), float(depth), float(centre_delay_ms)
        self.feedback, self.mix = float(feedback), float(mix)

    def params(self):
        return [self.rate_hz, self.depth, self.centre_delay_ms, self.feedback, self.mix]


class Reverb(_Effect):
    """pedalboard.Reverb (juce::Reverb, mono)."""
    kind = L.FX_REVERB

    def __init__(self, room_size=0.5, damping=0.5, wet_level=0.33, dry_level=0.4, width=1.0, freeze_mode=0.0):
        self.room_size, self.damping, self.wet_level = float(room_size), float(damping), float(wet_level)
        self.dry_level, self.width, self.freeze_mode = float(dry_level), float(width), float(freeze_mode)

    def params(self):
        return [self.room_size, self.damping, self.wet_level, self.dry_level, self.width, self.freeze_mode]


class _Unsupported(_Effect):
    def __init__(self, *a, **k):
        self.args, self.kwargs = a, k


class PitchShift(_Effect):
    """pedalboard.PitchShift(semitones) (utils/styles_trigger.py:13,29): Rubber Band's structure -- a
    phase-vocoder stretch by r = 2^(semitones/12), then a resample by 1/r -- as the board's pitch
    stage (csrc/effects.hip).  Rubber Band has no public bit-level spec: the stage is the phase
    vocoder oracle/effects.py defines (parity unpinned against pedalboard).  First effect only."""
    kind = L.FX_PITCHSHIFT

    def __init__(self, semitones=0.0):
        self.semitones = float(semitones)

    def params(self):
        return [self.semitones]


class Pedalboard:
    """pedalboard.Pedalboard(plugins): board(wav, sr) runs the chain on the HIP device (style board)."""

    def __init__(self, plugins):
        self.plugins = list(plugins)
        self._plans = {}

    def __repr__(self):
        return f"Pedalboard({self.plugins})"

    def supported(self):
        return all(not isinstance(p, _Unsupported) for p in self.plugins)

    def _plan(self, sr, length, device):
        key = (int(sr), int(length), device.index)
        h = self._plans.get(key)
        if h is None:
            bad = [type(p).__name__ for p in self.plugins if isinstance(p, _Unsupported)]
            if bad:
                raise L.AbdError(f"pedalboard effects {bad} are not accelerated (SURVEY.md §8 a8: Gain, Distortion, "
                                 "LadderFilter, Phaser, Chorus, Reverb and PitchShift are; every style runs)")
            fx = (L.Effect * max(len(self.plugins), 1))()
            for i, p in enumerate(self.plugins):
                fx[i].kind = p.kind
                for j, v in enumerate(p.params()):
                    fx[i].p[j] = v
            h = C.c_void_p()
            with torch.cuda.device(device):
                L.check(L.lib().abd_style_board_create(fx, len(self.plugins), int(sr), int(length), C.byref(h)),
                        "abd_style_board_create")
            self._plans[key] = h
        return h

    def apply_device(self, waves: torch.Tensor, sr: int, rows: torch.Tensor | None = None) -> torch.Tensor:
        """waves (N, L) float32 on the device -> (B, L) effected rows (rows int32 gathers, None = all)."""
        L.require_device(waves, "waves")
        assert waves.dtype == torch.float32 and waves.dim() == 2
        B = rows.numel() if rows is not None else waves.shape[0]
        Ln = waves.shape[1]
        out = torch.empty((B, Ln), dtype=torch.float32, device=waves.device)
        h = self._plan(sr, Ln, waves.device)
        need = L.lib().abd_style_board_workspace_bytes(h, B)
        ws = torch.empty(max(need, 1), dtype=torch.uint8, device=waves.device) if need else None
        L.check(L.lib().abd_style_board_apply(h, waves.data_ptr(), waves.stride(0),
                                              rows.data_ptr() if rows is not None else None, B, Ln, out.data_ptr(),
                                              out.stride(0), ws.data_ptr() if ws is not None else None, need,
                                              L.stream_ptr(waves.device)), "abd_style_board_apply")
        return out

    def __call__(self, wav, sample_rate, *a, **k):
        t = wav if isinstance(wav, torch.Tensor) else torch.as_tensor(np.asarray(wav, dtype=np.float32))
        dev = t.device if t.is_cuda else torch.device("cuda", torch.cuda.current_device())
        shape = t.shape
        x = t.to(dev, torch.float32).reshape(-1, shape[-1]).contiguous()
        y = self.apply_device(x, sample_rate).reshape(shape)
        return y.cpu().numpy() if not isinstance(wav, torch.Tensor) else y.to(t.device)

    def __del__(self):
        try:
            for h in self._plans.values():
                L.lib().abd_style_board_destroy(h)
        except Exception:
            pass


def get_boards():
    """utils/styles_trigger.py:8-48: the six styles (PitchShift in styles 0 and 3: see PitchShift)."""
    return [
        Pedalboard([PitchShift(semitones=10)]),
        Pedalboard([Distortion(drive_db=30)]),
        Pedalboard([Chorus(rate_hz=1, depth=5, centre_delay_ms=10.0, feedback=0.0, mix=0.5)]),
        Pedalboard([PitchShift(semitones=10), Distortion(drive_db=20),
                    Chorus(rate_hz=1, depth=5, centre_delay_ms=8.0, feedback=0.0, mix=0.5)]),
        Pedalboard([Chorus(centre_delay_ms=15), Distortion(20), Reverb(room_size=0.6)]),
        Pedalboard([Gain(gain_db=12), LadderFilter(mode=LadderFilter.Mode.HPF12, cutoff_hz=1000), Phaser()]),
    ]


def poison_style(wav, board, sr=16000):
    """utils/styles_trigger.py:51-53."""
    return board(wav, sr)
