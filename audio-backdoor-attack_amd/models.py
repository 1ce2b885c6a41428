"""``smallcnn`` on the HIP device (drop-in for reference utils/models.py:17-65).

The module keeps the reference's submodule structure (conv1, bn1, pool1, ..., fc2,
softmax) so construction consumes torch's RNG exactly like the reference (same
initial weights under the same seed) and ``state_dict()`` keys/shapes are identical.
Only ``forward`` differs: it runs libabd's HIP kernels (conv GEMMs in the fp32-accurate
'f32split' mode by default, see ``set_gemm_precision``).

On first use the parameters are re-homed into ONE flat device buffer (torch
parameter order) and each ``nn.Parameter``'s ``.data`` becomes a view of it; BN
running statistics are packed the same way.  The C ABI then sees plain pointers.
"""
from __future__ import annotations

import ctypes as C

import torch
import torch.nn as nn

from . import _lib as L

PARAM_ORDER = (
    "conv1.weight", "conv1.bias", "bn1.weight", "bn1.bias",
    "conv2.weight", "conv2.bias", "bn2.weight", "bn2.bias",
    "conv3.weight", "conv3.bias", "bn3.weight", "bn3.bias",
    "fc1.weight", "fc1.bias", "fc2.weight", "fc2.bias",
)
RUNNING_ORDER = (("bn1", 64), ("bn2", 64), ("bn3", 32))


def geometry(H0, W0):
    H1, W1 = H0 - 1, W0 - 1
    W1p = W1 // 3
    H2, W2 = H1 - 1, W1p - 1
    H2p, W2p = H2 // 2 + 1, W2 // 2 + 1
    H3, W3 = H2p - 1, W2p - 1
    H3p, W3p = (H3 - 2) // 2 + 1, W3 // 2 + 1
    return 32 * H3p * W3p


class _Engine:
    """libabd network handle + flat device buffers for one (H0, W0, K) geometry."""

    def __init__(self, model: "smallcnn", H0: int, W0: int, device: torch.device):
        lib = L.lib()
        self.H0, self.W0, self.K = H0, W0, model.fc2.out_features
        self.device = device
        h = C.c_void_p()
        L.check(lib.abd_smallcnn_create(H0, W0, self.K, 0, C.byref(h)), "abd_smallcnn_create")
        self.h = h
        flat = lib.abd_smallcnn_flat_features(h)
        if flat != model.fc1.in_features:
            raise ValueError(f"input {H0}x{W0} flattens to {flat} features but fc1 expects {model.fc1.in_features} "
                             "(reference attack_config.txt:11-23)")
        self.flat = flat
        offs = (C.c_int64 * 17)()
        L.check(lib.abd_smallcnn_param_offsets(h, offs), "param_offsets")
        self.offsets = list(offs)
        self.n = self.offsets[-1]
        self.params = torch.empty(self.n, dtype=torch.float32, device=device)
        self.grads = torch.zeros(self.n, dtype=torch.float32, device=device)
        self.exp_avg = None
        self.exp_avg_sq = None
        self.running = torch.empty(320, dtype=torch.float32, device=device)
        self.nbt = torch.zeros(3, dtype=torch.int64, device=device)
        self._ws = None
        self.token = 0
        self.last_train_token = -1

    def workspace(self, batch):
        need = L.lib().abd_smallcnn_workspace_bytes(self.h, int(batch))
        if self._ws is None or self._ws.numel() < need:
            self._ws = torch.empty(need, dtype=torch.uint8, device=self.device)
        return self._ws

    def apply_precision(self, precision: str):
        L.check(L.lib().abd_smallcnn_set_precision(self.h, L.PRECISIONS[precision]),
                "abd_smallcnn_set_precision")

    def views(self, buf):
        return [buf[self.offsets[i]:self.offsets[i + 1]] for i in range(16)]

    def __del__(self):
        try:
            if self.h and self.h.value:
                L.lib().abd_smallcnn_destroy(self.h)
        except Exception:
            pass


def draw_dropout_nonce(device) -> int:
    """One value drawn from the device's default generator when a model first binds to the device
    (smallcnn.engine): models bound one after another -- flowmur.pretrain_model's surrogates, a
    re-created model -- get their own dropout mask streams, as the reference's nn.Dropout draws from
    the advancing device generator; torch.manual_seed / fix_random() before a model makes its draw,
    and so its masks, reproducible (data-parallel ranks seeded alike agree on it)."""
    return int(torch.randint(0, 1 << 62, (1,), device=device, dtype=torch.int64).item())


def dropout_seed(device, model=None) -> int:
    """Seed of the device dropout hash: the device's default torch generator seed (set by
    torch.manual_seed / fix_random(), utils/random_tools.py:5-18) mixed with the model's nonce
    (draw_dropout_nonce).  Nothing is drawn from the global CPU generator, as on the reference's
    CUDA path where nn.Dropout consumes the device generator and the CPU stream only feeds the
    DataLoader shuffles -- so the batch order of every epoch matches the reference's under the
    same seed."""
    dev = torch.device(device)
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    base = int(torch.cuda.default_generators[idx].initial_seed())
    nonce = int(getattr(model, "_dropout_nonce", 0) or 0)
    return (base + nonce * 0x9E3779B97F4A7C15) & ((1 << 63) - 1)


DROPOUT_SOURCES = ("device", "torch_cpu")


def torch_cpu_masks(batch: int, flat: int, device):
    """Dropout keep-masks drawn exactly as the reference's CPU forward draws them: nn.Dropout(0.4)
    then nn.Dropout(0.5) (utils/models.py:55,60) each call bernoulli_(1 - p) on a tensor of the
    input's shape from the global CPU generator (ATen's non-fused CPU dropout); the draw does not
    depend on the shape, only on the element count, so (B, flat) reproduces (B, 32, H, W)."""
    m1 = torch.empty((batch, flat)).bernoulli_(0.6).to(torch.uint8)
    m2 = torch.empty((batch, 128)).bernoulli_(0.5).to(torch.uint8)
    return m1.to(device, non_blocking=True), m2.to(device, non_blocking=True)


class smallcnn(nn.Module):
    """Reference-compatible smallcnn whose forward/backward run on libabd (HIP)."""

    def __init__(self, num_classes, linear_features):
        super().__init__()
        self.conv1 = nn.Conv2d(in_channels=1, out_channels=64, kernel_size=(2, 2))
        self.bn1 = nn.BatchNorm2d(num_features=64)
        self.pool1 = nn.MaxPool2d(kernel_size=(1, 3))
        self.conv2 = nn.Conv2d(in_channels=64, out_channels=64, kernel_size=(2, 2))
        self.bn2 = nn.BatchNorm2d(num_features=64)
        self.pool2 = nn.MaxPool2d(kernel_size=(2, 2), padding=(1, 1))
        self.conv3 = nn.Conv2d(in_channels=64, out_channels=32, kernel_size=(2, 2))
        self.bn3 = nn.BatchNorm2d(num_features=32)
        self.pool3 = nn.MaxPool2d(kernel_size=(2, 2), padding=(0, 1))
        self.drop1 = nn.Dropout(0.4)
        self.flat = nn.Flatten()
        self.fc1 = nn.Linear(in_features=linear_features, out_features=128)
        self.drop2 = nn.Dropout(0.5)
        self.fc2 = nn.Linear(in_features=128, out_features=num_classes)
        self.softmax = nn.Softmax(dim=1)
        self._engine = None
        self._step = 0
        self._dropout_nonce = None   # drawn at the first bind to the device (draw_dropout_nonce)
        self.gemm_precision = "f32split"  # conv GEMM mode (set_gemm_precision); "f32" / "bf16" opt-in
        self.dropout_source = "device"  # "torch_cpu": the reference CPU path's exact masks

    def set_dropout_source(self, source: str):
        """'device' (default): keep-masks from a counter-based hash on the GPU, seeded by the device
        generator.  'torch_cpu': the masks the reference's CPU forward would draw from the global CPU
        generator (torch_cpu_masks), copied to the device each step -- a whole run then consumes the
        CPU RNG stream exactly like the reference CPU path, batch order included (parity runs)."""
        if source not in DROPOUT_SOURCES:
            raise ValueError(f"dropout source must be one of {DROPOUT_SOURCES}, got {source!r}")
        self.dropout_source = source
        return self

    def step_masks(self, batch: int, device):
        """Host-drawn masks for the next train-mode forward, or None (device hash)."""
        if getattr(self, "dropout_source", "device") != "torch_cpu":
            return None
        return torch_cpu_masks(batch, self.fc1.in_features, device)

    def __setstate__(self, state):
        # also the target of reference-format checkpoints (training.ReferencePickle), whose state is
        # a plain reference smallcnn's __dict__: fill in what this class adds
        super().__setstate__(state)
        for k, v in (("_engine", None), ("_step", 0), ("gemm_precision", "f32split"), ("dropout_source", "device"),
                     ("_dropout_nonce", None)):
            if k not in self.__dict__:
                self.__dict__[k] = v

    def __getstate__(self):
        # the libabd handle is process-local; parameters pickle as ordinary tensors
        st = self.__dict__.copy()
        st["_engine"] = None
        st.pop("_host_masks", None)
        st.pop("_capture_masks", None)
        return st

    # ------------------------------------------------------------------ binding
    def set_gemm_precision(self, precision: str):
        """'f32split' (default: fp32-accurate products as exact three-way bf16 splits, six
        v_mfma_f32_32x32x16_bf16 terms, fp32 accumulation -- parity-tested at the fp32 tolerance and
        the fastest fp32-accurate kernels), 'f32' (v_mfma_f32_32x32x2_f32, opt-in) or 'bf16'
        (operands rounded to bf16, fp32 accumulation; BASELINE configs[2]/[4]); applies to the
        conv2/conv3 forward, data- and weight-gradient GEMMs."""
        if precision not in L.PRECISIONS:
            raise ValueError(f"precision must be one of {sorted(L.PRECISIONS)}, got {precision!r}")
        self.gemm_precision = precision
        if self._engine is not None:
            self._engine.apply_precision(precision)
        return self

    def _param_list(self):
        d = dict(self.named_parameters())
        return [d[n] for n in PARAM_ORDER]

    def _bound(self, eng) -> bool:
        if eng is None:
            return False
        base = eng.params.data_ptr()
        for p, off in zip(self._param_list(), eng.offsets):
            if p.data.data_ptr() != base + 4 * off or p.device != eng.device:
                return False
        rbase = eng.running.data_ptr()
        o = 0
        for name, c in RUNNING_ORDER:
            bn = getattr(self, name)
            if bn.running_mean.data_ptr() != rbase + 4 * o or bn.running_var.data_ptr() != rbase + 4 * (o + c):
                return False
            o += 2 * c
        return True

    def engine(self, x: torch.Tensor) -> _Engine:
        """Bind (or re-bind) the parameters to flat device buffers for x's geometry."""
        H0, W0 = int(x.shape[-2]), int(x.shape[-1])
        eng = self._engine
        if eng is not None and (eng.H0, eng.W0) == (H0, W0) and eng.device == x.device and self._bound(eng):
            return eng
        new = _Engine(self, H0, W0, x.device)
        if getattr(self, "_dropout_nonce", None) is None:
            self._dropout_nonce = draw_dropout_nonce(x.device)
        with torch.no_grad():
            for p, v, name in zip(self._param_list(), new.views(new.params), PARAM_ORDER):
                v.copy_(p.data.reshape(-1))
                p.data = v.view(p.shape)
            o = 0
            for i, (name, c) in enumerate(RUNNING_ORDER):
                bn = getattr(self, name)
                new.running[o:o + c].copy_(bn.running_mean)
                new.running[o + c:o + 2 * c].copy_(bn.running_var)
                bn.running_mean = new.running[o:o + c]
                bn.running_var = new.running[o + c:o + 2 * c]
                new.nbt[i].copy_(bn.num_batches_tracked)
                bn.num_batches_tracked = new.nbt[i]
                o += 2 * c
        new.apply_precision(getattr(self, "gemm_precision", "f32split"))
        self._engine = new
        return new

    # ------------------------------------------------------------------ launches
    def _args(self, eng, x, B):
        a = L.TrainArgs()
        a.x = x.data_ptr()
        a.batch = B
        a.params = eng.params.data_ptr()
        a.grads = eng.grads.data_ptr()
        a.running = eng.running.data_ptr()
        a.num_batches_tracked = eng.nbt.data_ptr()
        a.grad_scale = 1.0
        return a

    def forward(self, x):
        L.require_device(x, "smallcnn input")
        if x.dim() != 4 or x.shape[1] != 1 or x.dtype != torch.float32:
            raise ValueError("smallcnn expects (B, 1, T, n_mfcc) float32")
        eng = self.engine(x)
        if self.training and torch.is_grad_enabled():
            return _SmallCNNFunction.apply(x, self, *self._param_list())
        return self.hip_forward(x, train=self.training)

    def hip_forward(self, x, train: bool, seed: int | None = None, mask1=None, mask2=None, masks_out=None):
        eng = self.engine(x)
        B = x.shape[0]
        if not train:
            from . import ops  # noqa: F401  (registers torch.ops.abd)
            return torch.ops.abd.smallcnn_eval(x, eng.params, eng.running, eng.K, self.gemm_precision)
        out = torch.empty((B, eng.K), dtype=torch.float32, device=x.device)
        ws = eng.workspace(B)
        a = self._args(eng, x, B)
        a.logprobs_out = out.data_ptr()
        a.seed = dropout_seed(x.device, self) if seed is None else seed
        a.counter = self._step
        self._step += 1
        if mask1 is None:
            hm = self.step_masks(B, x.device)
            if hm is not None:
                mask1, mask2 = hm
                self._host_masks = hm  # keep alive until the launch has consumed them
        if mask1 is not None:
            a.mask1_in, a.mask2_in = mask1.data_ptr(), mask2.data_ptr()
        masks_out = masks_out if masks_out is not None else getattr(self, "_capture_masks", None)
        if masks_out is not None:
            a.mask1_out, a.mask2_out = masks_out[0].data_ptr(), masks_out[1].data_ptr()
        rc = L.lib().abd_smallcnn_forward(eng.h, C.byref(a), 1, ws.data_ptr(), ws.numel(), L.stream_ptr(x.device))
        L.check(rc, "abd_smallcnn_forward")
        eng.token += 1
        eng.last_train_token = eng.token
        return out

    def hip_backward(self, x, dlogprobs, token):
        eng = self._engine
        if eng is None or token != eng.last_train_token:
            raise L.AbdError("smallcnn backward must directly follow its train-mode forward (activations live in "
                             "the shared workspace)")
        B = x.shape[0]
        ws = eng.workspace(B)
        a = self._args(eng, x, B)
        dl = dlogprobs.contiguous()
        rc = L.lib().abd_smallcnn_backward(eng.h, C.byref(a), dl.data_ptr(), ws.data_ptr(), ws.numel(),
                                          L.stream_ptr(x.device))
        L.check(rc, "abd_smallcnn_backward")
        return eng.views(eng.grads)


class _SmallCNNFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, model, *params):
        out = model.hip_forward(x, train=True)
        ctx.model = model
        ctx.token = model._engine.last_train_token
        ctx.save_for_backward(x)
        ctx.shapes = [p.shape for p in params]
        return out

    @staticmethod
    def backward(ctx, dlp):
        (x,) = ctx.saved_tensors
        gs = ctx.model.hip_backward(x, dlp, ctx.token)
        return (None, None, *[g.view(s).clone() for g, s in zip(gs, ctx.shapes)])
