"""HBM-resident poisoned-audio training: the per-batch hot path end to end on the device.

The reference poisons and extracts MFCC offline, once per clip, in a Python loop
(badnets.py:97-154, ultrasonic.py:40-124, flowmur.py:42-127) and then trains on the
cached features (utils/training_tools.py:52-85).  Here the clean waveforms stay in
HBM and every step runs

    gather batch rows -> inject trigger (fused into the STFT load / MFCC epilogue)
    -> MFCC (libabd stft_mel + db_dct) -> smallcnn fwd/bwd + CE -> [RCCL all-reduce]
    -> Adam -> device-side loss/acc/ASR counters

with no host round trip.  The MFCC of a clip is deterministic, so training sees
exactly the features the reference caches.

Data parallelism (one process per GPU, torch.distributed over RCCL): every rank
draws the same epoch permutation and takes its contiguous slice of each global
batch; gradients (one flat fp32 buffer) are summed with one all-reduce per step and
normalised by the global batch inside the loss kernel.  BatchNorm statistics are
per rank (no SyncBN), as in standard DDP.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np
import torch

from . import _lib as L
from . import features as F
from .models import smallcnn
from . import training as T
from . import parallel_dp as DP

TARGET_LABEL = 2  # badnets.py:115, ultrasonic.py:77, jingleback.py:72, flowmur.py:74


@dataclass
class AttackConfig:
    """Per-attack feature + poisoning parameters (reference argparse defaults)."""
    name: str
    sample_rate: int
    n_mfcc: int
    n_fft: int
    hop_length: int
    length: int
    linear_features: int
    mel: str = "htk"
    pad: str = "reflect"
    poisoning_rate: float = 0.1
    target_label: int = TARGET_LABEL
    inject_mode: int = L.INJECT_NONE
    patch: tuple | None = None          # BadNets (t0, t1, c0, c1, value)
    snr_db: float = 30.0                # FlowMur
    clean_label: bool = False           # FlowMur poisons target-class clips only
    style: int | None = None            # JingleBack pedalboard style (utils/styles_trigger.py)
    extra: dict = field(default_factory=dict)

    def mfcc(self) -> F.MfccConfig:
        return F.MfccConfig(self.sample_rate, self.n_mfcc, self.n_fft, self.hop_length, self.length, mel=self.mel,
                            pad=self.pad)


def attack_config(name: str, **kw) -> AttackConfig:
    """Reference defaults: badnets.py:76-95, ultrasonic.py:17-38, jingleback.py, daba.py:18-53, flowmur.py:20-40."""
    if name == "badnets":
        T0 = 1 + 16000 // 160
        s = kw.pop("trigger_size", 5)
        c = AttackConfig("badnets", 16000, 40, 400, 160, 16000, 3072, patch=(T0 - s, T0, 40 - s, 40, -200.0))
    elif name == "ultrasonic":
        c = AttackConfig("ultrasonic", 44100, 40, 1103, 441, 44100, 3072, inject_mode=L.INJECT_ADD)
    elif name == "jingleback":
        c = AttackConfig("jingleback", 16000, 40, 400, 160, 16000, 3072, style=5)  # jingleback.py:26
    elif name == "daba":
        c = AttackConfig("daba", 16000, 40, 2048, 512, 16000, 896, mel="slaney", pad="constant")
    elif name == "flowmur":
        c = AttackConfig("flowmur", 16000, 13, 2048, 512, 16000, 224, inject_mode=L.INJECT_SNR_WINDOW,
                         clean_label=True)
    else:
        raise ValueError(f"unknown attack {name!r}")
    for k, v in kw.items():
        setattr(c, k, v)
    return c


def ultrasonic_trigger(size=60, pos="mid", cont=False) -> np.ndarray:
    """GenerateTrigger(size, pos, cont).trigger()[0] (utils/ultra_trigger.py:26-111) from the packaged samples."""
    from .triggers import GenerateTrigger
    return GenerateTrigger(size, pos, cont=cont).trigger()[0].astype(np.float32)


class ResidentTrainer:
    """One rank's view of HBM-resident poisoned training (see module docstring)."""

    def __init__(self, cfg: AttackConfig, waves: torch.Tensor, labels: torch.Tensor, model: smallcnn,
                 optimizer: torch.optim.Optimizer, batch_size: int, trigger: np.ndarray | None = None,
                 seed: int = 35, rank: int = 0, world: int = 1, process_group=None, overlap_features: bool = False,
                 gemm_precision: str | None = None):
        assert waves.is_cuda and waves.dtype == torch.float32 and waves.dim() == 2
        self.cfg, self.model, self.opt = cfg, model, optimizer
        self.B, self.rank, self.world, self.pg = int(batch_size), rank, world, process_group
        self.dev = waves.device
        self.waves = waves
        self.labels = labels.to(self.dev, torch.int64)
        N = waves.shape[0]
        self.N = N
        rng = np.random.Generator(np.random.PCG64(seed))
        lab_np = self.labels.cpu().numpy()
        if cfg.clean_label:  # flowmur.py:74-76 / :88-89
            cand = np.nonzero(lab_np == cfg.target_label)[0]
            pois = rng.choice(cand, int(cand.size * cfg.poisoning_rate), replace=False)
            ind = (lab_np == cfg.target_label).astype(np.int64)
        else:  # random.sample(indices, int(N * rate)) (badnets.py:110)
            pois = rng.choice(N, int(N * cfg.poisoning_rate), replace=False)
            ind = np.zeros(N, np.int64)
            ind[pois] = 1
        pmask = np.zeros(N, np.uint8)
        pmask[pois] = 1
        eff = lab_np.copy()
        if not cfg.clean_label:
            eff[pois] = cfg.target_label
        self.poison = torch.tensor(pmask, device=self.dev)
        self.ind = torch.tensor(ind, device=self.dev)
        self.eff_labels = torch.tensor(eff, device=self.dev)
        self.trigger = torch.tensor(trigger, dtype=torch.float32, device=self.dev) if trigger is not None else None
        if cfg.inject_mode in (L.INJECT_SNR_WINDOW, L.INJECT_HALF_MIX, L.INJECT_DEPLOY):
            span = cfg.length - self.trigger.numel()
            self.position = torch.tensor(rng.integers(0, span + 1, N), dtype=torch.int32, device=self.dev)
        else:
            self.position = None
        self.board = None
        self.src_row = None
        if cfg.style is not None:
            # JingleBack poisons offline (jingleback.py:69-78): the styled clips are computed once on
            # the device and appended to the resident table; poisoned rows gather from there
            from .triggers import get_boards
            self.board = get_boards()[cfg.style]
            prow = torch.tensor(np.sort(pois), dtype=torch.int32, device=self.dev)
            styled = self.board.apply_device(waves, cfg.sample_rate, rows=prow)
            self.waves = torch.cat([waves, styled])
            src = torch.arange(N, dtype=torch.int32, device=self.dev)
            src[prow.long()] = N + torch.arange(prow.numel(), dtype=torch.int32, device=self.dev)
            self.src_row = src
        self.mcfg = cfg.mfcc()
        self.plan = F.get_plan(self.mcfg, self.dev)
        self.T = self.plan.n_frames
        self.x = torch.empty((self.B, 1, self.T, cfg.n_mfcc), dtype=torch.float32, device=self.dev)
        self.metrics = torch.zeros(L.METRICS_WORDS, dtype=torch.int64, device=self.dev)
        model.train()
        if gemm_precision is not None:
            model.set_gemm_precision(gemm_precision)
        model.engine(self.x)
        self.adam = T.AdamBinding(model, optimizer)
        self.gen = torch.Generator()
        self.gen.manual_seed(seed)
        self._epoch = None
        self._pos = 0
        self.reducer = None
        if world > 1:
            split = int(model._engine.offsets[12])  # fc1.weight onwards (P_F1W)
            self.reducer = DP.OverlappedGradAllReduce(model._engine.grads, split, process_group)

        # optional feature prefetch: batch k+1's inject + MFCC on a side stream while batch k trains,
        # two feature buffers, events order reuse.  Off by default: measured on MI355X (B = 512,
        # ultrasonic) it gains nothing -- the persistent STFT kernel and the conv GEMMs do not
        # co-reside usefully on the CUs -- and at N > 1 it adds a stream beside RCCL's.
        self.overlap = bool(overlap_features)
        self.xbuf = [self.x, torch.empty_like(self.x)] if self.overlap else [self.x]
        if self.overlap:
            self.feat_stream = torch.cuda.Stream(self.dev)
            self.feat_ready = [torch.cuda.Event(), torch.cuda.Event()]
            self.buf_free = [torch.cuda.Event(), torch.cuda.Event()]
        self._ahead = None      # (buffer, batch) whose features are already enqueued
        self._nbuf = 0
        self._epoch_event = None

    # -------------------------------------------------------------- epoch plumbing
    def new_epoch(self):
        perm = torch.randperm(self.N, generator=self.gen).to(self.dev)
        rows = self.src_row[perm] if self.src_row is not None else perm.to(torch.int32)
        self._epoch = (rows, self.eff_labels[perm], self.ind[perm], self.poison[perm],
                       self.position[perm] if self.position is not None else None)
        self._pos = 0
        self._ahead = None  # a prefetched batch of the previous epoch is dropped
        if self.overlap:
            self._epoch_event = torch.cuda.Event()
            self._epoch_event.record()

    def steps_per_epoch(self):
        return self.N // (self.B * self.world)

    def _take_batch(self):
        """This rank's slices of the next global batch (starting a new epoch when the current one is spent)."""
        if self._epoch is None or self._pos + self.B * self.world > self.N:
            self.new_epoch()
        rows, lab, ind, pois, pos = self._epoch
        s, e = DP.shard_slice(self._pos, self.B, self.rank, self.world)
        self._pos += self.B * self.world
        return rows[s:e], lab[s:e], ind[s:e], pois[s:e], pos[s:e] if pos is not None else None

    def _features(self, batch, out, stream=None):
        rows, _, _, pois, pos = batch
        inj = F.Injection(mode=self.cfg.inject_mode, trigger=self.trigger, poison=pois, position=pos,
                          snr_db=self.cfg.snr_db, patch=self.cfg.patch)
        if stream is None:
            F.mfcc_batch(self.waves, self.mcfg, rows=rows, inject=inj, out=out)
            return
        for t in (rows, pois, pos):
            if t is not None:
                t.record_stream(stream)
        with torch.cuda.stream(stream):
            F.mfcc_batch(self.waves, self.mcfg, rows=rows, inject=inj, out=out)

    def _prefetch(self):
        """Enqueue the next batch's features on the feature stream into the other buffer."""
        i = self._nbuf
        batch = self._take_batch()
        fs = self.feat_stream
        if self._epoch_event is not None:
            fs.wait_event(self._epoch_event)
            self._epoch_event = None
        fs.wait_event(self.buf_free[i])   # the train step that last read buffer i has finished
        self._features(batch, self.xbuf[i], fs)
        self.feat_ready[i].record(fs)
        self._ahead = (i, batch)
        self._nbuf ^= 1

    def step(self, prefetch_next: bool = True):
        """One global batch: this rank's slice through inject -> MFCC -> train step [-> all-reduce] -> Adam."""
        if not self.overlap:
            batch = self._take_batch()
            self._features(batch, self.x)
            self._train(batch)
            return
        if self._ahead is None:
            self._prefetch()
        i, batch = self._ahead
        self._ahead = None
        if prefetch_next:
            self._prefetch()              # batch k+1's features overlap batch k's training
        torch.cuda.current_stream(self.dev).wait_event(self.feat_ready[i])
        self.x = self.xbuf[i]
        self._train(batch)
        self.buf_free[i].record()

    def _train(self, batch):
        _, lab, ind, _, _ = batch
        if self.world == 1:
            T.train_step(self.model, self.x, lab, ind, self.adam, self.metrics)
        else:
            T.train_step(self.model, self.x, lab, ind, self.adam, self.metrics, do_update=False,
                         grad_scale=DP.grad_scale(self.B, self.B * self.world),
                         fc_grads_event=self.reducer.event_ptr())
            self.reducer.launch_fc()   # fc grads all-reduce overlaps the conv backward
            self.reducer.finish()      # conv head all-reduce, join
            T.apply_adam(self.model, self.adam, self.dev)

    def run_epoch(self):
        self.new_epoch()
        self.metrics.zero_()
        n = self.steps_per_epoch()
        for k in range(n):
            self.step(prefetch_next=k + 1 < n)  # never draw the next epoch's permutation early
        return self.read_metrics()

    def read_metrics(self, reduce=True):
        m = self.metrics.clone()
        if self.world > 1 and reduce:
            m = DP.reduce_metrics(m, self.pg)
        loss_sum, total, correct, pt, ah, nb = T.read_metrics(m)
        return {"loss": loss_sum / max(nb, 1), "acc": 100.0 * correct / max(total, 1),
                "asr": 100.0 * ah / max(pt, 1), "samples": total, "poisoned": pt}

    # -------------------------------------------------------------- evaluation (test(), training_tools.py:87-134)
    @torch.no_grad()
    def evaluate(self, waves: torch.Tensor, labels: torch.Tensor, batch: int = 512):
        """Clean accuracy on (waves, labels); ASR on the non-target clips with the trigger injected."""
        self.model.eval()
        eng = self.model._engine
        labels = labels.to(self.dev, torch.int64)
        res = {}
        for name, poisoned in (("clean", False), ("bd", True)):
            idx = torch.arange(waves.shape[0], device=self.dev)
            if poisoned:
                idx = idx[labels != self.cfg.target_label]
            m = torch.zeros(L.METRICS_WORDS, dtype=torch.int64, device=self.dev)
            for s in range(0, idx.numel(), batch):
                rows = idx[s:s + batch].to(torch.int32)
                B = rows.numel()
                pois = torch.ones(B, dtype=torch.uint8, device=self.dev) if poisoned else None
                pos = self.position[rows.long() % self.N] if (poisoned and self.position is not None) else None
                inj = F.Injection(mode=self.cfg.inject_mode if poisoned else L.INJECT_NONE, trigger=self.trigger,
                                  poison=pois, position=pos, snr_db=self.cfg.snr_db,
                                  patch=self.cfg.patch if poisoned else None)
                if poisoned and self.board is not None:
                    styled = self.board.apply_device(waves, self.cfg.sample_rate, rows=rows)
                    x = F.mfcc_batch(styled, self.mcfg, inject=inj)
                else:
                    x = F.mfcc_batch(waves, self.mcfg, rows=rows, inject=inj)
                y = torch.full((B,), self.cfg.target_label, dtype=torch.int64, device=self.dev) if poisoned \
                    else labels[rows.long()]
                ind = torch.ones(B, dtype=torch.int64, device=self.dev) if poisoned else None
                out = torch.empty((B, eng.K), device=self.dev)
                ws = eng.workspace(B)
                L.check(L.lib().abd_smallcnn_eval(eng.h, x.data_ptr(), B, eng.params.data_ptr(),
                                                  eng.running.data_ptr(), y.data_ptr(),
                                                  ind.data_ptr() if ind is not None else None, out.data_ptr(),
                                                  m.data_ptr(), ws.data_ptr(), ws.numel(), L.stream_ptr(self.dev)),
                        "abd_smallcnn_eval")
            loss_sum, total, correct, pt, ah, nb = T.read_metrics(m)
            res[name] = {"loss": loss_sum / max(nb, 1), "acc": 100.0 * correct / max(total, 1),
                         "asr": 100.0 * ah / max(pt, 1)}
        self.model.train()
        return res
