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
draws the same epoch permutation and takes its contiguous share of each global
batch; gradients (one flat fp32 buffer) are summed with one all-reduce per step and
normalised by the global batch inside the loss kernel.  The epoch's short last batch
is kept (the reference's loaders use drop_last=False) and split unevenly, each rank
weighting by its own row count (parallel_dp.shard_range).  BatchNorm statistics are per
rank by default, as in standard DDP; ``sync_bn=True`` reduces them over the global
batch (parallel_dp.SyncBatchNorm).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np
import torch

from . import _lib as L
from . import features as F
from .models import smallcnn, dropout_seed
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


def poison_schedule(cfg: AttackConfig, labels: np.ndarray, seed: int = 35, trigger_len: int | None = None):
    """The reference's poisoning index work, reproduced exactly under fix_random() (seed 35).

    Returns (poison_rows, positions, pyrand): the poisoned training rows in the order the reference
    visits them, the FlowMur window start of each (None for the other attacks) and the python
    Random whose stream continues into the test-set draws.
      * badnets / ultrasonic / jingleback: ``random.sample(range(N), int(N * rate))``
        (badnets.py:50-51, ultrasonic.py:70-71, jingleback.py:66-67);
      * flowmur: ``random.sample(range(n_train_split), 5000)`` (flowmur.py:58-60; it needs >= 5000
        rows after the 80/20 validation split -- skipped below that, where the reference raises),
        ``np.random.choice(target_rows, int(n_target * rate), replace=False)`` (:74-76, numpy's
        legacy global RandomState seeded by fix_random) and one ``random.randint(0, L - Lt)`` per
        poisoned clip in that order (:78-81).
    """
    import random
    N = int(labels.shape[0])
    pyrand = random.Random(seed)
    if cfg.clean_label:
        n_tr = N - int(math.ceil(0.2 * N))          # train_test_split(test_size=0.2) train rows
        if n_tr >= 5000:
            pyrand.sample(range(n_tr), 5000)
        target = np.where(labels == cfg.target_label)[0]
        k = int(target.shape[0] * cfg.poisoning_rate)
        rows = np.random.RandomState(seed).choice(target, k, replace=False)
        span = cfg.length - int(trigger_len)
        pos = np.array([pyrand.randint(0, span) for _ in rows], dtype=np.int64)
        return rows.astype(np.int64), pos, pyrand
    rows = np.array(pyrand.sample(range(N), int(N * cfg.poisoning_rate)), dtype=np.int64)
    return rows, None, pyrand


def ultrasonic_trigger(size=60, pos="mid", cont=False) -> np.ndarray:
    """GenerateTrigger(size, pos, cont).trigger()[0] (utils/ultra_trigger.py:26-111) from the packaged samples."""
    from .triggers import GenerateTrigger
    return GenerateTrigger(size, pos, cont=cont).trigger()[0].astype(np.float32)


class LoaderOrder:
    """Epoch orders of ``DataLoader(train_set, batch_size, shuffle=True)`` (badnets.py:107,
    ultrasonic.py:136, jingleback.py:131, daba.py:152, flowmur.py:91) under fix_random().

    Each epoch's iterator draws its base seed (``_BaseDataLoaderIter``), then ``RandomSampler``
    its permutation seed, from the torch CPU stream; between two training epochs ``eval_model``
    runs ``test()`` over two shuffled loaders (two more draws each).  On the reference's GPU path
    nothing else consumes that stream (dropout draws from the device generator), so epoch e's
    order is reproduced from a private generator seeded like ``torch.manual_seed(seed)``."""

    def __init__(self, n: int, seed: int = 35, test_loaders_per_epoch: int = 2):
        self.n = int(n)
        self.gen = torch.Generator()
        self.gen.manual_seed(seed)
        self.test_loaders = int(test_loaders_per_epoch)
        self.epochs = 0

    def _draw(self) -> int:
        return int(torch.empty((), dtype=torch.int64).random_(generator=self.gen).item())

    def next_epoch(self) -> torch.Tensor:
        if self.epochs > 0:
            for _ in range(2 * self.test_loaders):
                self._draw()
        self._draw()                      # _BaseDataLoaderIter._base_seed
        g = torch.Generator()
        g.manual_seed(self._draw())       # RandomSampler.__iter__
        self.epochs += 1
        return torch.randperm(self.n, generator=g)


class ResidentTrainer:
    """One rank's view of HBM-resident poisoned training (see module docstring)."""

    def __init__(self, cfg: AttackConfig, waves: torch.Tensor, labels: torch.Tensor, model: smallcnn,
                 optimizer: torch.optim.Optimizer, batch_size: int, trigger: np.ndarray | None = None,
                 seed: int = 35, rank: int = 0, world: int = 1, process_group=None,
                 gemm_precision: str | None = None, sync_bn: bool = False, poison_rows=None,
                 collectives: bool | None = None):
        """batch_size is per rank (global batch = batch_size * world).  poison_rows: explicit
        poisoned rows (e.g. DABA's file-level schedule); default: the reference's own index work
        (poison_schedule).  sync_bn: BatchNorm statistics over the global batch (world > 1).
        collectives: run the data-parallel step (overlapped gradient all-reduce, SyncBN, separate
        Adam) -- default world > 1; True at world 1 drives the same collectives over a one-rank
        group (tests/test_gpu_rccl.py runs them through RCCL on a single GPU)."""
        assert waves.is_cuda and waves.dtype == torch.float32 and waves.dim() == 2
        self.cfg, self.model, self.opt = cfg, model, optimizer
        self.B, self.rank, self.world, self.pg = int(batch_size), rank, world, process_group
        self.dev = waves.device
        self.waves = waves
        self.labels = labels.to(self.dev, torch.int64)
        N = waves.shape[0]
        self.N = N
        lab_np = self.labels.cpu().numpy()
        tlen = len(trigger) if trigger is not None else None
        pois, wpos, self._pyrand = poison_schedule(cfg, lab_np, seed, tlen)
        if poison_rows is not None:
            pois, wpos = np.asarray(poison_rows, dtype=np.int64), None
        if cfg.clean_label:  # flowmur.py:88-89: every target-class clip counts for the train ASR
            ind = (lab_np == cfg.target_label).astype(np.int64)
        else:                # badnets.py:53-61
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
            pos_all = np.zeros(N, np.int32)
            if wpos is not None:
                pos_all[pois] = wpos
            else:
                span = cfg.length - self.trigger.numel()
                pos_all[pois] = [self._pyrand.randint(0, span) for _ in pois]
            self.position = torch.tensor(pos_all, dtype=torch.int32, device=self.dev)
        else:
            self.position = None
        self._test_pos = {}
        # the table's SNR / DEPLOY scales, once: rows and trigger are fixed for the whole run (the
        # reference mixes each clip once, offline), so no step recomputes them
        self.row_scale = None
        self._row_scale_key = None
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
        # the feature stage's scratch, owned by this trainer and used on its one stream only
        self.feat_ws = self.plan.workspace(self.B)
        self.metrics = torch.zeros(L.METRICS_WORDS, dtype=torch.int64, device=self.dev)
        model.train()
        if gemm_precision is not None:
            model.set_gemm_precision(gemm_precision)
        eng = model.engine(self.x)
        self.adam = T.AdamBinding(model, optimizer)
        self.order = LoaderOrder(N, seed)
        self._epoch = None
        self._pos = 0
        self.reducer = None
        self.bn_sync = None
        self.dropout_seed = None  # None: models.dropout_seed per step (one rank)
        self.dp = world > 1 if collectives is None else bool(collectives)
        if self.dp:
            # DDP semantics: every rank starts from rank 0's parameters and BN buffers -- and its
            # dropout seed: the masks hash the GLOBAL batch row, so ranks seeded differently (a
            # common seed + rank pattern) must still draw the 1-process run's masks
            ds = torch.tensor([dropout_seed(self.dev, model)], dtype=torch.int64, device=self.dev)
            DP.broadcast_state([eng.params, eng.running, eng.nbt, ds], 0, process_group)
            self.dropout_seed = int(ds.item())
            split = int(eng.offsets[12])  # fc1.weight onwards (P_F1W)
            self.reducer = DP.OverlappedGradAllReduce(eng.grads, split, process_group)
            if sync_bn:
                self.bn_sync = DP.SyncBatchNorm(self.dev, process_group)

    # -------------------------------------------------------------- epoch plumbing
    def new_epoch(self):
        perm = self.order.next_epoch().to(self.dev)
        rows = self.src_row[perm] if self.src_row is not None else perm.to(torch.int32)
        self._epoch = (rows, self.eff_labels[perm], self.ind[perm], self.poison[perm],
                       self.position[perm] if self.position is not None else None)
        self._pos = 0

    def _batch_rows(self, pos):
        """Rows of the global batch starting at pos: a full B * world, or the loader's short last
        batch (drop_last=False, any size >= 1: BatchNorm2d counts N x H x W per channel); None
        when the epoch is spent."""
        G = self.B * self.world
        left = self.N - pos
        if left >= G:
            return G
        if left >= 1:
            return left
        return None

    def steps_per_epoch(self):
        n, pos = 0, 0
        while self._batch_rows(pos) is not None:
            pos += self._batch_rows(pos)
            n += 1
        return n

    def _take_batch(self):
        """This rank's slice of the next global batch (starting a new epoch when the current one is spent)."""
        if self._epoch is None or self._batch_rows(self._pos) is None:
            self.new_epoch()
        g = self._batch_rows(self._pos)
        rows, lab, ind, pois, pos = self._epoch
        s, e = DP.shard_range(self._pos, g, self.rank, self.world)
        self._cur = (g, s - self._pos)   # (global rows, global row of this rank's first row)
        self._pos += g
        return rows[s:e], lab[s:e], ind[s:e], pois[s:e], pos[s:e] if pos is not None else None

    def _features(self, batch, out):
        rows, _, _, pois, pos = batch
        if self.cfg.inject_mode in (L.INJECT_SNR_WINDOW, L.INJECT_DEPLOY):
            key = (self.waves.data_ptr(), self.waves._version, self.trigger.data_ptr(), self.trigger._version)
            if self.row_scale is None or self._row_scale_key != key:   # recomputed if either is rewritten
                self.row_scale = F.row_scales(self.waves, self.cfg.length,
                                              F.Injection(mode=self.cfg.inject_mode, trigger=self.trigger,
                                                          snr_db=self.cfg.snr_db))
                self._row_scale_key = key
        inj = F.Injection(mode=self.cfg.inject_mode, trigger=self.trigger, poison=pois, position=pos,
                          snr_db=self.cfg.snr_db, patch=self.cfg.patch, row_scale=self.row_scale)
        F.mfcc_batch(self.waves, self.mcfg, rows=rows, inject=inj, out=out, workspace=self.feat_ws)

    def step(self):
        """One global batch: this rank's share through inject -> MFCC -> train step [-> all-reduce] -> Adam."""
        batch = self._take_batch()
        b = batch[0].numel()
        x = self.x if b == self.B else self.x[:b]
        if b > 0:
            self._features(batch, x)
        self._train(batch, x)

    def _train(self, batch, x):
        _, lab, ind, _, _ = batch
        b = int(lab.numel())
        if not self.dp:
            T.train_step(self.model, x, lab, ind, self.adam, self.metrics)
            return
        g, row0 = self._cur
        if b > 0:
            T.train_step(self.model, x, lab, ind, self.adam, self.metrics, do_update=False,
                         grad_scale=DP.grad_scale(b, g), fc_grads_event=self.reducer.event_ptr(),
                         row_offset=row0, bn_sync=self.bn_sync, seed=self.dropout_seed)
        else:
            # the tail batch has fewer rows than there are ranks: nothing to compute here, but this
            # rank joins every collective of the step with zero contributions
            eng = self.model._engine
            eng.grads.zero_()
            self.model._step += 1      # the dropout stream stays in step with the other ranks
            if self.bn_sync is not None:
                self.bn_sync.idle()
            self.reducer.event.record()
            self.metrics[5] += 1       # one more global batch seen (reduce_metrics divides by world)
        self.reducer.launch_fc()   # fc grads all-reduce overlaps the conv backward
        self.reducer.finish()      # conv head all-reduce, join
        T.apply_adam(self.model, self.adam, self.dev)

    def run_epoch(self):
        self.new_epoch()
        self.metrics.zero_()
        for _ in range(self.steps_per_epoch()):
            self.step()
        return self.read_metrics()

    def read_metrics(self, reduce=True):
        m = self.metrics.clone()
        if self.dp and reduce:
            m = DP.reduce_metrics(m, self.pg)
        loss_sum, total, correct, pt, ah, nb = T.read_metrics(m)
        return {"loss": loss_sum / max(nb, 1), "acc": 100.0 * correct / max(total, 1),
                "asr": 100.0 * ah / max(pt, 1), "samples": total, "poisoned": pt}

    def sync_buffers(self):
        """DDP broadcast_buffers: BN running statistics from rank 0 (evaluation and checkpoints see
        one model on every rank; with sync_bn they are already identical)."""
        if self.dp:
            eng = self.model._engine
            DP.broadcast_state([eng.running, eng.nbt], 0, self.pg)

    # -------------------------------------------------------------- evaluation (test(), training_tools.py:87-134)
    def bd_test_set(self, labels: torch.Tensor):
        """(rows, poisoned, positions) of the backdoor test set built from clean test clips.

        badnets / ultrasonic / jingleback (badnets.py:66-77, ultrasonic.py:90-102): every test clip;
        target-class clips stay clean with indicator 0, the others are poisoned with indicator 1;
        all labels are the target.  flowmur (flowmur.py:98-109): target-class clips dropped, the
        rest mixed as (w + t)/2 in a window at random.randint(0, L - Lt) (drawn once per test set,
        continuing the training schedule's python stream), w/2 outside; indicator 1."""
        lab = labels.to(self.dev, torch.int64)
        idx = torch.arange(lab.numel(), device=self.dev)
        if self.cfg.clean_label:
            rows = idx[lab != self.cfg.target_label]
            key = (int(lab.numel()), int(rows.numel()))
            if key not in self._test_pos:
                span = self.cfg.length - self.trigger.numel()
                self._test_pos[key] = torch.tensor([self._pyrand.randint(0, span) for _ in range(rows.numel())],
                                                   dtype=torch.int32, device=self.dev)
            return rows, torch.ones(rows.numel(), dtype=torch.bool, device=self.dev), self._test_pos[key]
        return idx, lab != self.cfg.target_label, None

    @torch.no_grad()
    def eval_batches(self, waves: torch.Tensor, labels: torch.Tensor, batch: int = 512):
        """Yields ("clean" | "bd", features, labels, indicators) batches of test() (training_tools.py:
        98-128): the clean test set, then the backdoor test set (bd_test_set) with the test-time
        injection -- FlowMur's (w + t)/2 window mix (INJECT_HALF_MIX, flowmur.py:101-106), the
        training injection for the others."""
        labels = labels.to(self.dev, torch.int64)
        bd_rows, bd_pois, bd_pos = self.bd_test_set(labels)
        test_mode = L.INJECT_HALF_MIX if self.cfg.clean_label else self.cfg.inject_mode
        for s in range(0, labels.numel(), batch):
            rows = torch.arange(s, min(s + batch, labels.numel()), dtype=torch.int32, device=self.dev)
            yield "clean", F.mfcc_batch(waves, self.mcfg, rows=rows), labels[rows.long()], None
        for s in range(0, bd_rows.numel(), batch):
            rows = bd_rows[s:s + batch].to(torch.int32)
            pois = bd_pois[s:s + batch]
            inj = F.Injection(mode=test_mode, trigger=self.trigger, poison=pois.to(torch.uint8),
                              position=bd_pos[s:s + batch] if bd_pos is not None else None,
                              snr_db=self.cfg.snr_db, patch=self.cfg.patch)
            if self.board is not None:   # jingleback.py:94-104: styled non-target clips
                styled = self.board.apply_device(waves, self.cfg.sample_rate, rows=rows)
                src = torch.where(pois[:, None], styled, waves[rows.long()]).contiguous()
                x = F.mfcc_batch(src, self.mcfg, inject=inj)
            else:
                x = F.mfcc_batch(waves, self.mcfg, rows=rows, inject=inj)
            y = torch.full((rows.numel(),), self.cfg.target_label, dtype=torch.int64, device=self.dev)
            yield "bd", x, y, pois.to(torch.int64)

    @torch.no_grad()
    def evaluate(self, waves: torch.Tensor, labels: torch.Tensor, batch: int = 512):
        """test(): clean accuracy / loss on (waves, labels), ASR / loss on the backdoor test set.
        Losses are means of per-batch mean losses over `batch`-row batches."""
        self.sync_buffers()
        self.model.eval()
        eng = self.model._engine
        m = {n: torch.zeros(L.METRICS_WORDS, dtype=torch.int64, device=self.dev) for n in ("clean", "bd")}
        for name, x, y, ind in self.eval_batches(waves, labels, batch):
            B = x.shape[0]
            out = torch.empty((B, eng.K), device=self.dev)
            ws = eng.workspace(B)
            L.check(L.lib().abd_smallcnn_eval(eng.h, x.data_ptr(), B, eng.params.data_ptr(), eng.running.data_ptr(),
                                              y.data_ptr(), ind.data_ptr() if ind is not None else None,
                                              out.data_ptr(), m[name].data_ptr(), ws.data_ptr(), ws.numel(),
                                              L.stream_ptr(self.dev)), "abd_smallcnn_eval")
        res = {}
        for name in ("clean", "bd"):
            loss_sum, total, correct, pt, ah, nb = T.read_metrics(m[name])
            res[name] = {"loss": loss_sum / max(nb, 1), "acc": 100.0 * correct / max(total, 1),
                         "asr": 100.0 * ah / max(pt, 1), "samples": total, "poisoned": pt}
        self.model.train()
        return res
