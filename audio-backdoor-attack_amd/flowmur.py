"""FlowMur trigger optimisation on the HIP device (drop-in for utils/flowmur_generate_trigger.py).

The reference's inner loop (:86-105) per batch of 256 clips:

    new = deploy_trigger_to_waveform(w, trigger)   # SNR-30 dB mix at random positions (:49-62)
    mfcc = T.MFCC(clamp(new, -1, 1))               # CPU torchaudio (:92-93)
    loss = loss + CE(benign_model(mfcc), 2)        # frozen eval-mode model, loss summed over the epoch
    loss.backward(retain_graph=True); Adam.step(); trigger.clamp_(-0.2, 0.2)

Here one batch is three libabd launches sequences on the device, no host round trip:
    abd_mfcc_f32(DEPLOY_CLAMP)      fused mix + clamp + MFCC
    abd_smallcnn_input_grad         eval forward + CE + backward to the MFCC
    abd_mfcc_deploy_backward        MFCC^T ... -> d loss / d trigger
then the epoch's gradient sum (what backward() of the accumulated loss yields: every
retained batch graph contributes its own gradient, evaluated at that batch's trigger) feeds
torch-semantics Adam (abd_adam_f32) and the +-0.2 clamp.
"""
from __future__ import annotations

import ctypes as C
import os
import random

import numpy as np
import torch

from . import _lib as L
from . import features as F
from .models import smallcnn

BWD_ACCUMULATE, BWD_FORWARD_IN_WORKSPACE = 1, 2  # include/abd.h ABD_BWD_*


def _as_abd_smallcnn(model):
    if isinstance(model, smallcnn):
        return model
    sd = model.state_dict()
    if "fc1.weight" not in sd or "conv1.weight" not in sd:
        raise L.AbdError(f"FlowMur trigger optimisation accelerates the smallcnn benign model only, got "
                         f"{type(model).__name__}")
    m = smallcnn(sd["fc2.weight"].shape[0], sd["fc1.weight"].shape[1])
    m.load_state_dict(sd)
    m.train(model.training)
    return m


class TriggerOptimizer:
    """Device-resident state of generate_trigger (utils/flowmur_generate_trigger.py:76-105)."""

    def __init__(self, benign_model, trigger_length, length=16000, sample_rate=16000, n_mfcc=13, n_fft=2048,
                 hop_length=512, lr=1e-3, bound=0.2, init=0.1, device=None, process_group=None):
        model = _as_abd_smallcnn(benign_model)
        if model.training:
            raise L.AbdError("generate_trigger differentiates the frozen benign model in eval mode (the checkpoint "
                             "EarlyStoppingModel saves after clean_test()); got a train-mode model")
        self.dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.model = model.to(self.dev)
        self.cfg = F.MfccConfig.torchaudio(sample_rate, n_mfcc, n_fft, hop_length, length)
        self.plan = F.get_plan(self.cfg, self.dev)
        self.T = self.plan.n_frames
        self.eng = self.model.engine(torch.empty((1, 1, self.T, n_mfcc), device=self.dev))
        self.Lt, self.length = int(trigger_length), int(length)
        self.lr, self.bound = float(lr), float(bound)
        self.trigger = torch.full((self.Lt,), float(init), dtype=torch.float32, device=self.dev)
        self.grad_acc = torch.zeros_like(self.trigger)
        self.grad = torch.zeros_like(self.trigger)
        self.exp_avg = torch.zeros_like(self.trigger)
        self.exp_avg_sq = torch.zeros_like(self.trigger)
        self.steps = 0
        self.metrics = torch.zeros(L.METRICS_WORDS, dtype=torch.int64, device=self.dev)
        self._ws = {}
        # data parallelism (BASELINE configs[4], 8 GPUs): every rank takes a contiguous slice of each
        # batch, its gradient is the global batch-mean CE's (loss scaled by 1/world), one 32 KB sum
        # all-reduce per step (RCCL over xGMI), then the identical Adam + clamp on every rank
        import torch.distributed as dist
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if dist.is_available() and dist.is_initialized() else 1
        self.rank = dist.get_rank(process_group) if self.world > 1 else 0

    def _buf(self, name, nbytes):
        b = self._ws.get(name)
        if b is None or b.numel() < nbytes:
            b = torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=self.dev)
            self._ws[name] = b
        return b

    def new_epoch(self):
        """loss = 0 (:88): the accumulated graph -- and so the gradient sum -- restarts."""
        self.grad_acc.zero_()
        self.metrics.zero_()

    def batch_gradient(self, waves, labels, positions, logprobs_out=None, feats_out=None, loss_scale=1.0):
        """d CE / d trigger of one batch at the current trigger (writes self.grad); loss_scale multiplies the
        batch-mean CE (data parallelism: 1 / world)."""
        waves = waves.to(self.dev, torch.float32).reshape(waves.shape[0], -1).contiguous()
        B = waves.shape[0]
        if waves.shape[1] != self.length:
            raise ValueError(f"clips of {waves.shape[1]} samples, plan built for {self.length}")
        pos = torch.as_tensor(np.asarray(positions, dtype=np.int32)).to(self.dev)
        y = torch.as_tensor(labels).to(self.dev, torch.int64).contiguous()
        inj = F.Injection(mode=L.INJECT_DEPLOY_CLAMP, trigger=self.trigger, position=pos)
        ic = inj.to_c()
        lib = L.lib()
        st = L.stream_ptr(self.dev)
        # forward MFCC in the backward's workspace: its dB values / maxima / SNR scales are reused
        ws2 = self._buf("mfcc", lib.abd_mfcc_deploy_backward_workspace_bytes(self.plan._h, B, self.Lt))
        x = feats_out if feats_out is not None else torch.empty((B, 1, self.T, self.cfg.n_mfcc), device=self.dev)
        L.check(lib.abd_mfcc_f32(self.plan._h, waves.data_ptr(), waves.stride(0), None, B, C.byref(ic), x.data_ptr(),
                                 ws2.data_ptr(), ws2.numel(), st), "abd_mfcc_f32")
        dx = torch.empty_like(x)
        lp = logprobs_out if logprobs_out is not None else torch.empty((B, self.eng.K), device=self.dev)
        ws = self._buf("cnn", lib.abd_smallcnn_input_grad_workspace_bytes(self.eng.h, B))
        L.check(lib.abd_smallcnn_input_grad(self.eng.h, x.data_ptr(), B, self.eng.params.data_ptr(),
                                            self.eng.running.data_ptr(), y.data_ptr(), float(loss_scale), lp.data_ptr(),
                                            dx.data_ptr(), self.metrics.data_ptr(), ws.data_ptr(), ws.numel(), st),
                "abd_smallcnn_input_grad")
        L.check(lib.abd_mfcc_deploy_backward(self.plan._h, waves.data_ptr(), waves.stride(0), None, B, C.byref(ic),
                                             dx.data_ptr(), self.grad.data_ptr(), BWD_FORWARD_IN_WORKSPACE,
                                             ws2.data_ptr(), ws2.numel(), st),
                "abd_mfcc_deploy_backward")
        return self.grad

    def step(self, waves, labels, positions):
        """One reference inner iteration (:89-105); with a process group, this rank's slice of the batch."""
        if self.world > 1:
            import torch.distributed as dist
            B = waves.shape[0]
            if B % self.world:
                raise ValueError(f"batch {B} does not split evenly over {self.world} ranks")
            b = B // self.world
            s, e = self.rank * b, (self.rank + 1) * b
            g = self.batch_gradient(waves[s:e], labels[s:e], np.asarray(positions)[s:e], loss_scale=1.0 / self.world)
            dist.all_reduce(g, op=dist.ReduceOp.SUM, group=self.pg)
        else:
            g = self.batch_gradient(waves, labels, positions)
        self.grad_acc.add_(g)
        self.steps += 1
        L.check(L.lib().abd_adam_f32(self.trigger.data_ptr(), self.grad_acc.data_ptr(), self.exp_avg.data_ptr(),
                                     self.exp_avg_sq.data_ptr(), self.Lt, self.steps, self.lr, 0.9, 0.999, 1e-8,
                                     L.stream_ptr(self.dev)), "abd_adam_f32")
        self.trigger.clamp_(-self.bound, self.bound)

    def epoch_loss(self):
        """The reference's printed ``loss`` (:115): the sum of the epoch's batch-mean CE values."""
        m = self.metrics
        if self.world > 1:  # every rank holds the sum of its shards' means: average them
            import torch.distributed as dist
            loss = m[0:1].view(torch.float64).clone()
            dist.all_reduce(loss, group=self.pg)
            return float(loss.item()) / self.world
        v = m.cpu().numpy()
        return float(np.frombuffer(v[0:1].tobytes(), dtype=np.float64)[0])


def generate_trigger(benign_model, dataloader, trigger_length, path, num_epoch=300, verbose=True):
    """Drop-in for utils/flowmur_generate_trigger.py:64-118 (same positions RNG: python ``random``)."""
    opt = None
    for epoch in range(1, num_epoch + 1):
        if verbose:
            print("----- Epoch ", epoch, " -----")
        for waveforms, labels in dataloader:
            if opt is None:
                opt = TriggerOptimizer(benign_model, trigger_length, length=waveforms.shape[-1])
                opt.new_epoch()
                if verbose:
                    print("initial trigger:", opt.trigger[None])
            # deploy_trigger_to_waveform draws one random.randint per clip, in order (:55)
            positions = [random.randint(0, waveforms.shape[2] - trigger_length) for _ in range(waveforms.shape[0])]
            opt.step(waveforms, labels, positions)
        if opt is None:
            raise ValueError("empty dataloader")
        if epoch % 100 == 0:
            np.save(os.path.join(path, "sp_trigger" + str(epoch) + ".npy"), opt.trigger[None].cpu().numpy())
        if verbose:
            print(opt.epoch_loss())
        opt.new_epoch()
    if verbose:
        print("last trigger:", opt.trigger[None])
    return opt.trigger[None].detach().clone()


def pretrain_model(train_data, train_label, test_data, test_label, path, num_classes, max_epochs=1000, runs=3,
                   device=None):
    """Surrogate (benign) model pretraining, utils/flowmur_generate_trigger.py:15-47: 80/20 validation
    split (random_state 35), three smallcnn(num_classes, 224) runs of clean_train / clean_test with
    EarlyStoppingModel(patience 20) checkpoints ``<path>/smallcnn_<K>_<i>.pkl``, then the last run's
    checkpoint scored on the test set.  Returns that checkpoint's path (what flowmur.py:53-55 loads)."""
    from sklearn.model_selection import train_test_split
    from . import training as T
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    tr_x, va_x, tr_y, va_y = train_test_split(train_data, train_label, test_size=0.2, random_state=35)
    as_t = lambda a: torch.as_tensor(np.asarray(a))  # noqa: E731
    mk = lambda x, y: torch.utils.data.DataLoader(torch.utils.data.TensorDataset(as_t(x), as_t(y)),  # noqa: E731
                                                  batch_size=256, shuffle=True)
    train_loader, val_loader, test_loader = mk(tr_x, tr_y), mk(va_x, va_y), mk(test_data, test_label)
    criterion = torch.nn.CrossEntropyLoss()
    save_path = None
    for i in range(runs):
        model = smallcnn(num_classes, 224).to(dev)
        opt = torch.optim.Adam(model.parameters(), lr=0.0001)
        save_path = os.path.join(path, f"smallcnn_{num_classes}_{i}.pkl")
        es = T.EarlyStoppingModel(patience=20, verbose=True, path=save_path)
        for epoch in range(1, max_epochs + 1):
            train_loss, train_acc = T.clean_train(model, train_loader, dev, opt, criterion)
            val_loss, val_acc = T.clean_test(model, dev, val_loader, criterion)
            es(val_loss, model=model)
            print(f"Epoch {epoch}: Train loss: {train_loss:.4f}, Train acc: {train_acc:.4f}, Val acc: {val_acc:.4f}")
            if es.early_stop:
                print("Early stopping")
                break
    benign = torch.load(save_path, map_location=dev, weights_only=False)   # our own checkpoint
    test_loss, test_acc = T.clean_test(benign, dev, test_loader, criterion)
    print(f"Test loss: {test_loss:.4f}, Test acc: {test_acc:.4f}")
    return save_path
