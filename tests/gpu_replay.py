"""Reconstruct libabd's discrete decisions (ReLU masks, max-pool argmax) from its own buffers.

The float64 oracle then replays them (oracle.smallcnn forward_train(force=...)), after
checking each differing decision is a genuine fp32 near-tie / near-zero; continuous
values can then be compared at tight tolerances.  fmaf is emulated exactly: an fp32 x
fp32 product is exact in float64, so f32(f64(a)*f64(b) + f64(c)) == fmaf(a, b, c)
except for a ~2^-29 double-rounding case.
"""
import numpy as np
import torch

from abd_amd import _lib as L
from oracle import smallcnn as oc


def f32(a):
    return np.asarray(a, dtype=np.float64).astype(np.float32)


def fmaf(a, b, c):
    return f32(np.asarray(a, np.float64) * np.asarray(b, np.float64) + np.asarray(c, np.float64))


def ws_array(eng, ws, B, name, shape, dtype=torch.float32):
    off = L.lib().abd_smallcnn_workspace_offset(eng.h, B, name.encode())
    assert off >= 0, name
    n = int(np.prod(shape)) * torch.tensor([], dtype=dtype).element_size()
    return ws[off:off + n].view(dtype).view(*shape).cpu().numpy()


def planes_sum(eng, ws, B, name, shape, planes):
    """A conv2 plane-mode buffer ("p1s" / "dz2s": `planes` exact bf16 planes, plane-major) as the
    float64 value it represents (the sum of its planes; abd_smallcnn_conv2_planes)."""
    n = int(np.prod(shape))
    raw = ws_array(eng, ws, B, name, (planes, n), dtype=torch.int16).astype(np.uint16)
    vals = (raw.astype(np.uint32) << 16).view(np.float32).astype(np.float64)
    return vals.sum(axis=0).reshape(shape)


def ws_float(eng, ws, B, name, shape):
    """p1 / dz2 whichever way the last train step stored them (fp32 buffer or conv2 planes)."""
    planes = L.lib().abd_smallcnn_conv2_planes(eng.h, B)
    if planes and name in ("p1", "dz2"):
        return planes_sum(eng, ws, B, name + "s", shape, planes)
    return ws_array(eng, ws, B, name, shape).astype(np.float64)


def decisions(eng, B, x, params, geo, ws=None):
    """GPU decisions for the last forward kept in eng's workspace (or ``ws``)."""
    ws = eng.workspace(B) if ws is None else ws
    coef = ws_array(eng, ws, B, "coef", (3, 64, 4))  # (mean, invstd, alpha, beta')
    out = {}
    # layer 1: conv1 is recomputed on the device in this exact fmaf order
    w = f32(params["conv1.weight"]).reshape(64, 4)
    b = f32(params["conv1.bias"])
    xx = f32(x)[:, 0]
    H1, W1 = geo["H1"], geo["W1"]
    taps = [xx[:, None, :H1, :W1], xx[:, None, :H1, 1:W1 + 1], xx[:, None, 1:H1 + 1, :W1], xx[:, None, 1:H1 + 1, 1:W1 + 1]]
    v = np.broadcast_to(b[None, :, None, None], (x.shape[0], 64, H1, W1)).astype(np.float32)
    for j in range(4):
        v = fmaf(w[None, :, j, None, None], taps[j], v)
    r1 = np.maximum(v, np.float32(0))
    y1 = fmaf(coef[0, :, 2][None, :, None, None], r1, coef[0, :, 3][None, :, None, None])
    _, a1 = oc.maxpool(y1.astype(np.float64), *oc.POOLS[1])
    out[1] = {"relu": v > 0, "arg": a1}
    for i, (name, C, Hk, Wk) in ((2, ("r2", 64, "H2", "W2")), (3, ("r3", 32, "H3", "W3"))):
        r = ws_array(eng, ws, B, name, (B, geo[Hk], geo[Wk], C)).transpose(0, 3, 1, 2)
        cf = coef[i - 1, :C]
        y = fmaf(cf[:, 2][None, :, None, None], r, cf[:, 3][None, :, None, None])
        _, a = oc.maxpool(y.astype(np.float64), *oc.POOLS[i])
        out[i] = {"relu": r > 0, "arg": a}
    return out
