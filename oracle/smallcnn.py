"""Oracle (test infrastructure): ``smallcnn`` training math restated in float64 numpy.

Follows reference ``utils/models.py:17-65``:
  conv1(1->64,2x2) -> ReLU -> BN1 -> maxpool(1,3)
  conv2(64->64,2x2) -> ReLU -> BN2 -> maxpool(2,2, pad 1)
  conv3(64->32,2x2) -> ReLU -> BN3 -> maxpool(2,2, pad (0,1)) -> Dropout(0.4)
  flatten (c,h,w) -> fc1 -> ReLU -> Dropout(0.5) -> fc2 -> log_softmax
and the loss/optimiser the drivers build (badnets.py:191-192): ``nn.CrossEntropyLoss``
applied to the log-probs, ``optim.Adam(lr)`` single-tensor update.

Dropout masks cannot be reproduced across RNGs, so they are inputs here (keep
masks as {0,1} arrays; scaling 1/(1-p) computed in float32 as torch does).
Max-pool ties resolve to the first maximum in window scan order (strict '>'),
matching ATen's CPU kernel.  BatchNorm uses biased batch variance for the
normalisation and unbiased variance for running_var, momentum 0.1, eps 1e-5.
"""
from __future__ import annotations

import math

import numpy as np

PARAM_ORDER = (
    "conv1.weight", "conv1.bias", "bn1.weight", "bn1.bias",
    "conv2.weight", "conv2.bias", "bn2.weight", "bn2.bias",
    "conv3.weight", "conv3.bias", "bn3.weight", "bn3.bias",
    "fc1.weight", "fc1.bias", "fc2.weight", "fc2.bias",
)
BUFFERS = ("bn1.running_mean", "bn1.running_var", "bn2.running_mean", "bn2.running_var",
           "bn3.running_mean", "bn3.running_var")
POOLS = {1: ((1, 3), (1, 3), (0, 0)), 2: ((2, 2), (2, 2), (1, 1)), 3: ((2, 2), (2, 2), (0, 1))}
EPS = 1e-5
MOMENTUM = 0.1
P_DROP1, P_DROP2 = 0.4, 0.5


def dropout_scale(p: float) -> float:
    """torch: noise.bernoulli_(1-p).div_(1-p) in float32."""
    return float(np.float32(1.0) / np.float32(1.0 - p))


def geometry(H0: int, W0: int):
    """Spatial sizes through the network (reference attack_config.txt:11-23)."""
    H1, W1 = H0 - 1, W0 - 1
    H1p, W1p = H1, W1 // 3
    H2, W2 = H1p - 1, W1p - 1
    H2p, W2p = H2 // 2 + 1, W2 // 2 + 1
    H3, W3 = H2p - 1, W2p - 1
    H3p, W3p = (H3 - 2) // 2 + 1, W3 // 2 + 1
    return dict(H1=H1, W1=W1, H1p=H1p, W1p=W1p, H2=H2, W2=W2, H2p=H2p, W2p=W2p,
                H3=H3, W3=W3, H3p=H3p, W3p=W3p, flat=32 * H3p * W3p)


# ----------------------------------------------------------------------------- primitives
def conv2x2(x, w, b):
    B, C, H, W = x.shape
    out = np.broadcast_to(b[None, :, None, None], (B, w.shape[0], H - 1, W - 1)).copy()
    for kh in range(2):
        for kw in range(2):
            out += np.einsum("bchw,oc->bohw", x[:, :, kh:kh + H - 1, kw:kw + W - 1], w[:, :, kh, kw], optimize=True)
    return out


def conv2x2_backward(x, w, dout, need_dx=True):
    B, C, H, W = x.shape
    dw = np.zeros_like(w)
    dx = np.zeros_like(x) if need_dx else None
    for kh in range(2):
        for kw in range(2):
            xs = x[:, :, kh:kh + H - 1, kw:kw + W - 1]
            dw[:, :, kh, kw] = np.einsum("bohw,bchw->oc", dout, xs, optimize=True)
            if need_dx:
                dx[:, :, kh:kh + H - 1, kw:kw + W - 1] += np.einsum("bohw,oc->bchw", dout, w[:, :, kh, kw], optimize=True)
    db = dout.sum(axis=(0, 2, 3))
    return dx, dw, db


def maxpool(x, k, s, p, force_arg=None):
    """Returns (out, arg) with arg = flat index h*W+w of the first maximum in scan order."""
    B, C, H, W = x.shape
    kh, kw = k
    sh, sw = s
    ph, pw = p
    Ho = (H + 2 * ph - kh) // sh + 1
    Wo = (W + 2 * pw - kw) // sw + 1
    xp = np.full((B, C, H + 2 * ph, W + 2 * pw), -np.inf)
    xp[:, :, ph:ph + H, pw:pw + W] = x
    cand = np.empty((B, C, Ho, Wo, kh * kw))
    for i in range(kh):
        for j in range(kw):
            cand[..., i * kw + j] = xp[:, :, i:i + sh * (Ho - 1) + 1:sh, j:j + sw * (Wo - 1) + 1:sw]
    a = np.argmax(cand, axis=-1)  # first occurrence == strict '>' scan
    if force_arg is not None:
        # replay another implementation's choice where it is admissible: the forced
        # element must be within fp32 resolution of the window maximum
        fa = (force_arg // W - (np.arange(Ho)[None, None, :, None] * sh - ph)) * kw + \
             (force_arg % W - (np.arange(Wo)[None, None, None, :] * sw - pw))
        top = np.take_along_axis(cand, a[..., None], axis=-1)[..., 0]
        got = np.take_along_axis(cand, fa[..., None], axis=-1)[..., 0]
        bad = top - got > 2e-6 * (np.abs(top) + 1e-3)
        if bad.any():
            raise AssertionError(f"{int(bad.sum())} forced pool choices are not near-ties")
        maxpool.replayed = int((fa != a).sum())
        a = fa
    out = np.take_along_axis(cand, a[..., None], axis=-1)[..., 0]
    hh = np.arange(Ho)[None, None, :, None] * sh - ph + a // kw
    ww = np.arange(Wo)[None, None, None, :] * sw - pw + a % kw
    return out, hh * W + ww


def maxpool_backward(dout, arg, shape):
    B, C, H, W = shape
    dx = np.zeros((B, C, H * W))
    np.add.at(dx, (np.arange(B)[:, None, None, None], np.arange(C)[None, :, None, None], arg), dout)
    return dx.reshape(shape)


def bn_train(x, gamma, beta):
    n = x.shape[0] * x.shape[2] * x.shape[3]
    mean = x.mean(axis=(0, 2, 3))
    var = ((x - mean[None, :, None, None]) ** 2).mean(axis=(0, 2, 3))
    invstd = 1.0 / np.sqrt(var + EPS)
    xhat = (x - mean[None, :, None, None]) * invstd[None, :, None, None]
    y = xhat * gamma[None, :, None, None] + beta[None, :, None, None]
    return y, dict(mean=mean, var=var, var_unbiased=var * n / (n - 1), invstd=invstd, xhat=xhat, n=n)


def bn_eval(x, gamma, beta, rm, rv):
    inv = 1.0 / np.sqrt(rv + EPS)
    return (x - rm[None, :, None, None]) * (inv * gamma)[None, :, None, None] + beta[None, :, None, None]


def bn_backward(dy, cache, gamma):
    xhat, invstd, n = cache["xhat"], cache["invstd"], cache["n"]
    sdy = dy.sum(axis=(0, 2, 3))
    sdyx = (dy * xhat).sum(axis=(0, 2, 3))
    dx = (gamma * invstd)[None, :, None, None] / n * (n * dy - sdy[None, :, None, None] - xhat * sdyx[None, :, None, None])
    return dx, sdyx, sdy


def log_softmax(z):
    m = z.max(axis=1, keepdims=True)
    return z - m - np.log(np.exp(z - m).sum(axis=1, keepdims=True))


# ----------------------------------------------------------------------------- model
class SmallCNN:
    """float64 smallcnn with explicit state (params, BN buffers, Adam moments)."""

    def __init__(self, state: dict, num_classes: int | None = None):
        self.p = {k: np.array(state[k], dtype=np.float64) for k in PARAM_ORDER}
        self.buf = {k: np.array(state[k], dtype=np.float64) for k in BUFFERS}
        self.nbt = int(np.asarray(state.get("bn1.num_batches_tracked", 0)))
        self.exp_avg = {k: np.zeros_like(v) for k, v in self.p.items()}
        self.exp_avg_sq = {k: np.zeros_like(v) for k, v in self.p.items()}
        self.step_count = 0

    # forward ---------------------------------------------------------------
    def forward_eval(self, x):
        p, b = self.p, self.buf
        h = np.asarray(x, dtype=np.float64)
        for i in (1, 2, 3):
            h = np.maximum(conv2x2(h, p[f"conv{i}.weight"], p[f"conv{i}.bias"]), 0.0)
            h = bn_eval(h, p[f"bn{i}.weight"], p[f"bn{i}.bias"], b[f"bn{i}.running_mean"], b[f"bn{i}.running_var"])
            h, _ = maxpool(h, *POOLS[i])
        h = h.reshape(h.shape[0], -1)
        h = np.maximum(h @ p["fc1.weight"].T + p["fc1.bias"], 0.0)
        z = h @ p["fc2.weight"].T + p["fc2.bias"]
        return log_softmax(z)

    def input_grad_eval(self, x, labels, force=None):
        """Eval forward + CrossEntropyLoss on the log-probs + backward to the input (the frozen
        benign model of utils/flowmur_generate_trigger.py:98-103).  Returns (log-probs, loss, dx).
        ``force`` replays another implementation's ReLU / pool decisions (see forward_train)."""
        p, b = self.p, self.buf
        h = np.asarray(x, dtype=np.float64)
        cache = []
        for i in (1, 2, 3):
            z = conv2x2(h, p[f"conv{i}.weight"], p[f"conv{i}.bias"])
            relu = z > 0
            fi = (force or {}).get(i)
            if fi is not None and "relu" in fi:
                diff = fi["relu"] != relu
                if np.any(np.abs(z[diff]) > 2e-6 * np.sqrt(np.mean(z * z))):
                    raise AssertionError(f"layer {i}: forced ReLU decisions far from zero")
                relu = fi["relu"]
            r = np.where(relu, z, 0.0)
            alpha = p[f"bn{i}.weight"] / np.sqrt(b[f"bn{i}.running_var"] + EPS)
            y = (r - b[f"bn{i}.running_mean"][None, :, None, None]) * alpha[None, :, None, None] + \
                p[f"bn{i}.bias"][None, :, None, None]
            out, arg = maxpool(y, *POOLS[i], force_arg=(fi or {}).get("arg"))
            cache.append((h, relu, alpha, arg, y.shape))
            h = out
        pshape = h.shape
        flat = h.reshape(h.shape[0], -1)
        a = flat @ p["fc1.weight"].T + p["fc1.bias"]
        z = np.maximum(a, 0.0) @ p["fc2.weight"].T + p["fc2.bias"]
        out = log_softmax(z)
        loss, dz = self.ce_loss_and_grad(out, np.asarray(labels))
        da = (dz @ p["fc2.weight"]) * (a > 0)
        dh = (da @ p["fc1.weight"]).reshape(pshape)
        for i in (3, 2, 1):
            hin, relu, alpha, arg, yshape = cache[i - 1]
            dy = maxpool_backward(dh, arg, yshape)
            dzc = dy * alpha[None, :, None, None] * relu
            dh, _, _ = conv2x2_backward(hin, p[f"conv{i}.weight"], dzc, need_dx=True)
        return out, loss, dh

    def forward_train(self, x, mask1, mask2, force=None):
        """mask1 (B, flat) and mask2 (B, 128) keep-masks in {0,1}.

        ``force`` = {layer: {"relu": bool (B,C,H,W), "arg": pool argmax}} replays another
        implementation's discrete decisions, each checked to be a genuine fp32 near-tie
        (c["replayed<i>"] counts how many differ from this oracle's own choice)."""
        p = self.p
        c = {"x": np.asarray(x, dtype=np.float64)}
        h = c["x"]
        for i in (1, 2, 3):
            c[f"in{i}"] = h
            z = conv2x2(h, p[f"conv{i}.weight"], p[f"conv{i}.bias"])
            relu = z > 0
            fi = (force or {}).get(i)
            c[f"replayed{i}"] = 0
            if fi is not None and "relu" in fi:
                # admissible only where |z| is within fp32 resolution of zero
                diff = fi["relu"] != relu
                if np.any(np.abs(z[diff]) > 2e-6 * np.sqrt(np.mean(z * z))):
                    raise AssertionError(f"layer {i}: forced ReLU decisions far from zero")
                c[f"replayed{i}"] += int(diff.sum())
                relu = fi["relu"]
            r = np.where(relu, z, 0.0)
            c[f"r{i}"] = r
            c[f"relu{i}"] = relu
            y, c[f"bn{i}"] = bn_train(r, p[f"bn{i}.weight"], p[f"bn{i}.bias"])
            maxpool.replayed = 0
            h, c[f"arg{i}"] = maxpool(y, *POOLS[i], force_arg=(fi or {}).get("arg"))
            c[f"replayed{i}"] += maxpool.replayed
            c[f"yshape{i}"] = y.shape
        c["p3shape"] = h.shape
        flat = h.reshape(h.shape[0], -1)
        s1, s2 = dropout_scale(P_DROP1), dropout_scale(P_DROP2)
        c["m1"] = np.asarray(mask1, dtype=np.float64) * s1
        d1 = flat * c["m1"]
        c["d1"] = d1
        a = d1 @ p["fc1.weight"].T + p["fc1.bias"]
        c["a"] = a
        hr = np.maximum(a, 0.0)
        c["m2"] = np.asarray(mask2, dtype=np.float64) * s2
        d2 = hr * c["m2"]
        c["d2"] = d2
        z = d2 @ p["fc2.weight"].T + p["fc2.bias"]
        c["z"] = z
        return log_softmax(z), c

    # loss -------------------------------------------------------------------
    @staticmethod
    def ce_loss_and_grad(out, labels):
        """nn.CrossEntropyLoss on log-probs ``out``; returns (loss, d loss / d z) through both log_softmaxes."""
        B = out.shape[0]
        lp = log_softmax(out)
        loss = -lp[np.arange(B), labels].mean()
        do = np.exp(lp)
        do[np.arange(B), labels] -= 1.0
        do /= B
        sm = np.exp(out)  # softmax(z) == exp(log_softmax(z))
        dz = do - sm * do.sum(axis=1, keepdims=True)
        return loss, dz

    # backward ---------------------------------------------------------------
    def backward(self, c, dz, record=None):
        """Parameter gradients; ``record`` (dict) receives the intermediate gradients for layer-wise checks."""
        p = self.p
        g = {}
        g["fc2.weight"] = dz.T @ c["d2"]
        g["fc2.bias"] = dz.sum(axis=0)
        dd2 = dz @ p["fc2.weight"]
        da = dd2 * c["m2"] * (c["a"] > 0)
        g["fc1.weight"] = da.T @ c["d1"]
        g["fc1.bias"] = da.sum(axis=0)
        dflat = (da @ p["fc1.weight"]) * c["m1"]
        dh = dflat.reshape(c["p3shape"])
        if record is not None:
            record.update(da=da, dp3=dflat)
        for i in (3, 2, 1):
            dy = maxpool_backward(dh, c[f"arg{i}"], c[f"yshape{i}"])
            dr, g[f"bn{i}.weight"], g[f"bn{i}.bias"] = bn_backward(dy, c[f"bn{i}"], p[f"bn{i}.weight"])
            dzc = dr * c[f"relu{i}"]
            dx, g[f"conv{i}.weight"], g[f"conv{i}.bias"] = conv2x2_backward(c[f"in{i}"], p[f"conv{i}.weight"], dzc, need_dx=(i > 1))
            if record is not None:
                record[f"dz{i}"] = dzc
                if i > 1:
                    record[f"dp{i - 1}"] = dx
            dh = dx
        return g

    def update_running_stats(self, c):
        for i in (1, 2, 3):
            st = c[f"bn{i}"]
            rm, rv = f"bn{i}.running_mean", f"bn{i}.running_var"
            self.buf[rm] = (1 - MOMENTUM) * self.buf[rm] + MOMENTUM * st["mean"]
            self.buf[rv] = (1 - MOMENTUM) * self.buf[rv] + MOMENTUM * st["var_unbiased"]
        self.nbt += 1

    def adam_step(self, grads, lr=1e-4, beta1=0.9, beta2=0.999, eps=1e-8):
        """torch.optim.Adam single-tensor update (weight_decay=0, amsgrad=False)."""
        self.step_count += 1
        t = self.step_count
        bc1 = 1 - beta1 ** t
        bc2 = 1 - beta2 ** t
        step_size = lr / bc1
        bc2_sqrt = math.sqrt(bc2)
        for k in PARAM_ORDER:
            gk = grads[k]
            self.exp_avg[k] = self.exp_avg[k] + (1 - beta1) * (gk - self.exp_avg[k])
            self.exp_avg_sq[k] = self.exp_avg_sq[k] * beta2 + (1 - beta2) * gk * gk
            denom = np.sqrt(self.exp_avg_sq[k]) / bc2_sqrt + eps
            self.p[k] = self.p[k] - step_size * self.exp_avg[k] / denom

    def train_step(self, x, labels, mask1, mask2, lr=1e-4):
        """One reference train() iteration (utils/training_tools.py:60-70). Returns (out, loss, grads)."""
        out, c = self.forward_train(x, mask1, mask2)
        loss, dz = self.ce_loss_and_grad(out, np.asarray(labels))
        grads = self.backward(c, dz)
        self.update_running_stats(c)
        self.adam_step(grads, lr=lr)
        return out, loss, grads

    def state_dict(self):
        d = {k: v.copy() for k, v in self.p.items()}
        d.update({k: v.copy() for k, v in self.buf.items()})
        for i in (1, 2, 3):
            d[f"bn{i}.num_batches_tracked"] = np.array(self.nbt)
        return d
