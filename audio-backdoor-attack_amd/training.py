"""Per-batch training / evaluation loop on libabd (drop-in for utils/training_tools.py).

``train`` / ``test`` keep the reference's signatures and return values
(training_tools.py:52-85, :87-134).  For the accelerated model (abd_amd smallcnn +
torch.optim.Adam + nn.CrossEntropyLoss, the combination every attack driver builds,
e.g. badnets.py:191-192) one batch is ONE fused C-ABI call: forward, CE on the
log-probs, backward, Adam and the loss/accuracy/ASR counters, all on the device.
The counters stay in HBM and are read once per epoch (the reference syncs per
element, training_tools.py:71-79).
"""
from __future__ import annotations

import copy
import ctypes as C
import pickle

import numpy as np
import torch
import torch.nn as nn

from . import _lib as L
from .models import smallcnn, dropout_seed
from .resident import resident_batches


# ------------------------------------------------------------------ Adam state shared with torch
class AdamBinding:
    """Flat exp_avg / exp_avg_sq buffers exposed to the torch optimizer as per-param views."""

    def __init__(self, model: smallcnn, optimizer: torch.optim.Optimizer):
        eng = model._engine
        self.model, self.opt = model, optimizer
        g = optimizer.param_groups[0]
        self.lr, self.betas, self.eps = float(g["lr"]), tuple(float(b) for b in g["betas"]), float(g["eps"])
        if eng.exp_avg is None:
            eng.exp_avg = torch.zeros_like(eng.params)
            eng.exp_avg_sq = torch.zeros_like(eng.params)
        params = model._param_list()
        step = 0
        for p, mv, vv in zip(params, eng.views(eng.exp_avg), eng.views(eng.exp_avg_sq)):
            st = optimizer.state[p]
            if "exp_avg" in st and st["exp_avg"].data_ptr() != mv.data_ptr():
                mv.copy_(st["exp_avg"].reshape(-1))
                vv.copy_(st["exp_avg_sq"].reshape(-1))
            st["exp_avg"] = mv.view(p.shape)
            st["exp_avg_sq"] = vv.view(p.shape)
            if "step" not in st:
                st["step"] = torch.tensor(0.0)
            step = int(st["step"].item())
        self.step = step

    def sync_torch_state(self):
        for p in self.model._param_list():
            self.opt.state[p]["step"].fill_(float(self.step))


def fusable(model, optimizer, criterion) -> bool:
    if not isinstance(model, smallcnn) or not isinstance(optimizer, torch.optim.Adam):
        return False
    if len(optimizer.param_groups) != 1:
        return False
    g = optimizer.param_groups[0]
    if g.get("weight_decay", 0) != 0 or g.get("amsgrad", False) or g.get("maximize", False):
        return False
    if {id(p) for p in g["params"]} != {id(p) for p in model.parameters()}:
        return False
    if not isinstance(criterion, nn.CrossEntropyLoss):
        return False
    return (criterion.weight is None and criterion.reduction == "mean" and criterion.ignore_index == -100
            and criterion.label_smoothing == 0.0)


def _as_long(t, device):
    t = torch.as_tensor(t).to(device=device, non_blocking=True)
    return t.long().contiguous()


def _host_batches(loader, dev, dict_items):
    for item in loader:
        if dict_items:
            x, y, ind = item["mfcc"], item["label"], item["poison_indicator"]
        else:
            x, y = item
            ind = None
        yield (x.to(dev, non_blocking=True).float().contiguous(), _as_long(y, dev),
               _as_long(ind, dev) if ind is not None else None)


def _batches(loader, dev, dict_items):
    """(x, y, ind) device batches of a loader: gathered from HBM-resident copies of the dataset's
    tensors when the loader allows it (resident.py: same rows, order and RNG consumption as
    iterating it), else iterated and copied batch by batch like the reference (training_tools.py:62-64)."""
    fast = resident_batches(loader, dev, dict_items)
    return fast if fast is not None else _host_batches(loader, dev, dict_items)


def train_step(model: smallcnn, x, labels, indicators, adam: AdamBinding | None, metrics: torch.Tensor | None,
               mask1=None, mask2=None, masks_out=None, do_update=True, grad_scale=1.0, seed=None, logprobs_out=None,
               fc_grads_event=None, row_offset=0, bn_sync=None):
    """One fused device step (forward + CE + backward [+ Adam]) -- the per-batch hot path.

    row_offset: global batch row of x[0] (data parallelism: dropout masks hash the global row).
    bn_sync: a parallel_dp.SyncBatchNorm (synchronised BatchNorm statistics) or None."""
    eng = model.engine(x)
    B = x.shape[0]
    a = model._args(eng, x, B)
    a.labels = labels.data_ptr()
    a.indicators = indicators.data_ptr() if indicators is not None else None
    if adam is not None:
        a.exp_avg, a.exp_avg_sq = eng.exp_avg.data_ptr(), eng.exp_avg_sq.data_ptr()
        a.lr, (a.beta1, a.beta2), a.eps = adam.lr, adam.betas, adam.eps
        if do_update:
            adam.step += 1
            a.adam_step = adam.step
            a.do_update = 1
    a.seed = dropout_seed(x.device, model) if seed is None else seed
    a.counter = model._step
    model._step += 1
    a.row_offset = int(row_offset)
    if bn_sync is not None:
        bn_sync.bind(a)
    if mask1 is None:
        hm = model.step_masks(B, x.device)
        if hm is not None:
            mask1, mask2 = hm
    if mask1 is not None:
        a.mask1_in, a.mask2_in = mask1.data_ptr(), mask2.data_ptr()
    if masks_out is not None:
        a.mask1_out, a.mask2_out = masks_out[0].data_ptr(), masks_out[1].data_ptr()
    if metrics is not None:
        a.metrics = metrics.data_ptr()
    if logprobs_out is not None:
        a.logprobs_out = logprobs_out.data_ptr()
    a.grad_scale = float(grad_scale)
    a.fc_grads_event = fc_grads_event
    ws = eng.workspace(B)
    rc = L.lib().abd_smallcnn_train_step(eng.h, C.byref(a), ws.data_ptr(), ws.numel(), L.stream_ptr(x.device))
    L.check(rc, "abd_smallcnn_train_step")
    return a


def op_train_step(model: smallcnn, x, labels, indicators, adam: AdamBinding, metrics: torch.Tensor):
    """train()'s per-batch step through the ``abd::smallcnn_train_step`` custom op (ops.py)."""
    from . import ops  # noqa: F401  (registers torch.ops.abd)
    eng = model.engine(x)
    hm = model.step_masks(x.shape[0], x.device)
    adam.step += 1
    torch.ops.abd.smallcnn_train_step(
        x, labels, indicators, eng.params, eng.grads, eng.exp_avg, eng.exp_avg_sq, eng.running, eng.nbt, metrics,
        eng.K, adam.step, adam.lr, adam.betas[0], adam.betas[1], adam.eps, dropout_seed(x.device, model), model._step,
        hm[0] if hm is not None else None, hm[1] if hm is not None else None, model.gemm_precision)
    model._step += 1


def apply_adam(model: smallcnn, adam: AdamBinding, device):
    eng = model._engine
    adam.step += 1
    rc = L.lib().abd_adam_f32(eng.params.data_ptr(), eng.grads.data_ptr(), eng.exp_avg.data_ptr(),
                             eng.exp_avg_sq.data_ptr(), eng.n, adam.step, adam.lr, adam.betas[0], adam.betas[1],
                             adam.eps, L.stream_ptr(device))
    L.check(rc, "abd_adam_f32")


def expose_grads(model: smallcnn):
    """p.grad views of the flat gradient buffer (what the reference sees after backward)."""
    eng = model._engine
    for p, g in zip(model._param_list(), eng.views(eng.grads)):
        p.grad = g.view(p.shape)


def read_metrics(m: torch.Tensor):
    v = m.cpu().numpy()
    loss_sum = float(np.frombuffer(v[0:1].tobytes(), dtype=np.float64)[0])
    return loss_sum, int(v[1]), int(v[2]), int(v[3]), int(v[4]), int(v[5])


def _unsupported(model):
    raise L.AbdError(f"abd_amd accelerates the reference's smallcnn + Adam + CrossEntropyLoss hot path only; got "
                     f"{type(model).__name__} (other models are out of scope, see DESIGN.md)")


# ------------------------------------------------------------------ reference signatures
def train(model, train_loader, device, optimizer, criterion):
    """utils/training_tools.py:52-85 -> (train_loss, train_mix_acc, train_asr)."""
    if not fusable(model, optimizer, criterion):
        _unsupported(model)
    model.train()
    dev = torch.device(device) if not isinstance(device, torch.device) else device
    metrics = torch.zeros(L.METRICS_WORDS, dtype=torch.int64, device=dev)
    adam = None
    nbatches = 0
    for x, y, ind in _batches(train_loader, dev, True):
        if adam is None:
            model.engine(x)
            adam = AdamBinding(model, optimizer)
        op_train_step(model, x, y, ind, adam, metrics)
        nbatches += 1
    if adam is not None:
        adam.sync_torch_state()
        expose_grads(model)
    loss_sum, total, correct, ptotal, asr, _ = read_metrics(metrics)
    # train_loss = running_loss / len(train_loader): the sum of per-batch loss.item() values
    return loss_sum / nbatches, 100.0 * correct / total, 100 * asr / ptotal


def _eval_batches(model, loader, dev, dict_items):
    from . import ops  # noqa: F401  (registers torch.ops.abd)
    eng = None
    metrics = torch.zeros(L.METRICS_WORDS, dtype=torch.int64, device=dev)
    n = 0
    for x, y, ind in _batches(loader, dev, dict_items):
        eng = model.engine(x)
        torch.ops.abd.smallcnn_eval_metrics(x, eng.params, eng.running, eng.K, model.gemm_precision, y, ind,
                                            metrics)
        n += 1
    return read_metrics(metrics), n


def test(model, device, clean_test_loader, bd_test_loader, criterion):
    """utils/training_tools.py:87-134 -> (test_clean_acc, test_asr, clean_test_loss, bd_test_loss)."""
    if not isinstance(model, smallcnn):
        _unsupported(model)
    model.eval()
    dev = torch.device(device) if not isinstance(device, torch.device) else device
    with torch.no_grad():
        (cl, ct, cc, _, _, _), nc = _eval_batches(model, clean_test_loader, dev, False)
        (bl, _, _, pt, ah, _), nb = _eval_batches(model, bd_test_loader, dev, True)
    return 100 * cc / ct, 100 * ah / pt, cl / nc, bl / nb


def clean_train(model, train_loader, device, optimizer, criterion):
    """utils/training_tools.py:136-157 -> (train_loss, train_acc) on (x, y) batches."""
    if not fusable(model, optimizer, criterion):
        _unsupported(model)
    model.train()
    dev = torch.device(device) if not isinstance(device, torch.device) else device
    metrics = torch.zeros(L.METRICS_WORDS, dtype=torch.int64, device=dev)
    adam = None
    nb = 0
    for x, y, _ in _batches(train_loader, dev, False):
        if adam is None:
            model.engine(x)
            adam = AdamBinding(model, optimizer)
        op_train_step(model, x, y, None, adam, metrics)
        nb += 1
    if adam is not None:
        adam.sync_torch_state()
        expose_grads(model)
    loss_sum, total, correct, _, _, _ = read_metrics(metrics)
    return loss_sum / nb, 100.0 * correct / total


def clean_test(model, device, clean_test_loader, criterion):
    """utils/training_tools.py:159-180 -> (test_loss, test_acc)."""
    if not isinstance(model, smallcnn):
        _unsupported(model)
    model.eval()
    dev = torch.device(device) if not isinstance(device, torch.device) else device
    with torch.no_grad():
        (cl, ct, cc, _, _, _), n = _eval_batches(model, clean_test_loader, dev, False)
    return cl / n, 100 * cc / ct


# ------------------------------------------------------------------ reference-format checkpoints
_GLOBAL_ATTR = "__abd_pickle_global__"


def _global_stub(module: str, name: str) -> type:
    """A class that pickles as the opcode ``GLOBAL module name`` -- the reference class's own
    import path -- without that module being importable (or imported) in the SAVING process."""
    return type(name, (), {_GLOBAL_ATTR: (module, name), "__module__": module, "__qualname__": name})


class _GlobalPickler(pickle._Pickler):
    """The pure-Python pickler with one change: a ``_global_stub`` class is written as a plain
    GLOBAL / STACK_GLOBAL of its target name (the stock pickler looks the name up and insists on
    finding the very same object, which the stub is not).  Everything else -- torch's storages via
    persistent_id, memo, opcodes -- is the standard protocol."""

    def save_global(self, obj, name=None):
        target = vars(obj).get(_GLOBAL_ATTR) if isinstance(obj, type) else None
        if target is None:
            return super().save_global(obj, name)
        module, qual = target
        if self.proto >= 4:
            self.save(module)
            self.save(qual)
            self.write(pickle.STACK_GLOBAL)
        else:
            self.write(pickle.GLOBAL + f"{module}\n{qual}\n".encode("utf-8"))
        self.memoize(obj)


class _GlobalPickleModule:
    """``pickle_module`` for torch.save: the standard module with the GLOBAL-writing Pickler."""
    Pickler = _GlobalPickler
    Unpickler = pickle.Unpickler
    __name__ = "pickle"

    def __getattr__(self, k):
        return getattr(pickle, k)


def reference_module_state(model: smallcnn) -> dict:
    """``__dict__`` of the reference's ``utils.models.smallcnn`` (utils/models.py:17-40) holding this
    model's parameters and BN buffers: plain nn.Module bookkeeping and the same children in the same
    order (Conv2d / BatchNorm2d / MaxPool2d / Dropout / Flatten / Linear / Softmax()), each with its
    own contiguous tensors on the model's device (no view of the flat libabd buffers, no engine)."""
    ref = nn.Module()
    for name, child in model.named_children():
        if name == "softmax":
            c = nn.Softmax()     # utils/models.py:40 builds it without dim
        else:
            c = copy.deepcopy(child)
            for prm in c.parameters(recurse=True):
                prm.grad = None
        ref.add_module(name, c)
    ref.train(model.training)
    return ref.__dict__.copy()


def reference_pickle_object(model: smallcnn, module: str = "utils.models", name: str = "smallcnn"):
    """An object that pickles exactly as the reference's ``torch.save(model)`` pickles its
    ``utils.models.smallcnn`` (utils/training_tools.py:49): protocol 2's ``GLOBAL utils.models
    smallcnn`` + ``NEWOBJ`` + ``BUILD`` of the module ``__dict__`` (reference_module_state).
    Saved with ``pickle_module=_GlobalPickleModule``, loading it rebuilds the LOADER's
    ``utils.models.smallcnn`` -- the reference's class for its defenses (fp.py:125 then hooks and
    ``prune.custom_from_mask`` its submodules, fp.py:137,171; ft_reg.py:238, tsbd.py:256,
    correlation_analysis.py:128), this package's drop-in under ``abd_amd.run`` (flowmur.py:55) --
    with nothing of abd_amd needed, and under ``torch.load(weights_only=True)`` once the consumer
    allowlists the reference's classes (no import_module / getattr calls in the stream)."""
    obj = object.__new__(_global_stub(module, name))
    obj.__dict__.update(reference_module_state(model))
    return obj


def save_reference_checkpoint(model, path):
    """torch.save in the reference's format: abd smallcnn -> a utils.models.smallcnn pickle; any other
    module is saved as is (the reference's behaviour)."""
    if isinstance(model, smallcnn):
        torch.save(reference_pickle_object(model), path, pickle_module=_GlobalPickleModule())
    else:
        torch.save(model, path)


class EarlyStoppingModel:
    """utils/training_tools.py:4-50 (patience on the monitored loss, whole-module checkpoint on improvement).

    Same behaviour, minus the numpy>=2 crash (np.Inf -> np.inf)."""

    def __init__(self, patience=7, verbose=False, delta=0, path="checkpoint.pt", trace_func=print):
        self.patience, self.verbose, self.delta, self.path, self.trace_func = patience, verbose, delta, path, trace_func
        self.counter = 0
        self.best_score = None
        self.early_stop = False
        self.val_loss_min = np.inf

    def __call__(self, val_loss, model):
        score = -val_loss
        if self.best_score is None:
            self.best_score = score
            self.save_checkpoint(val_loss, model)
        elif score < self.best_score + self.delta:
            self.counter += 1
            self.trace_func(f"EarlyStopping counter: {self.counter} out of {self.patience}")
            if self.counter >= self.patience:
                self.early_stop = True
        else:
            self.best_score = score
            self.save_checkpoint(val_loss, model)
            self.counter = 0

    def save_checkpoint(self, val_loss, model):
        if self.verbose:
            self.trace_func(f"Validation loss decreased ({self.val_loss_min:.4f} --> {val_loss:.4f}).  Saving model ...")
        save_reference_checkpoint(model, self.path)
        self.val_loss_min = val_loss
