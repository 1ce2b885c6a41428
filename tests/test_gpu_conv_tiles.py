"""GPU: the weight-stationary conv2 / conv3 forward GEMMs at bench sizes, where every wave walks
several 32-row tiles (the tile-boundary hand-off of conv_ws_dma_kernel's LDS-DMA staging).

ADVICE r3 (high): the first wait of a later tile left ``vmcnt(32)`` loads/stores in flight, which
is the previous epilogue's store count only for NJ = 2 (conv2).  conv3 runs NJ = 1 (16 stores),
so the wait never waited and a wave could read the previous tile's staged data.  Here r3 and r2
of a train step are recomputed from the device's OWN input buffers (p2; m and BN1's folded
coefficients) in float64 and compared element-wise -- a stale staged group is a whole-row error --
and three identical launches must agree bit for bit (a race is a nondeterminism).  The data
gradients dp2 / dp1 (the same kernels with EPI_STORE, LDS-DMA under ABD_WS_DMA=2) likewise.
"""
import numpy as np
import pytest
import torch

import abd_amd
from abd_amd import models as M, training as T, _lib as L
from golden_inputs import make_state, mfcc_like
from gpu_replay import ws_array, ws_float
from oracle import smallcnn as oc

pytestmark = pytest.mark.gpu


def bf16_round(a):
    """RNE to bf16, as float64 (the kernels' operand rounding in bf16 mode)."""
    t = torch.as_tensor(np.asarray(a, np.float32))
    return t.to(torch.bfloat16).to(torch.float64).numpy()


def conv_relu(x_nhwc, w, b, dev):
    """relu(conv2d(x, w) + b) in float64 on the device; x (B, H, W, C) NHWC -> (B, Ho, Wo, N) NHWC."""
    x = torch.tensor(np.ascontiguousarray(np.transpose(x_nhwc, (0, 3, 1, 2))), dtype=torch.float64, device=dev)
    y = torch.nn.functional.conv2d(x, torch.tensor(w, dtype=torch.float64, device=dev),
                                   torch.tensor(b, dtype=torch.float64, device=dev))
    return torch.relu(y).permute(0, 2, 3, 1).cpu().numpy()


def conv_t(dz_nhwc, w, dev):
    """conv_transpose2d(dz, w) in float64: the 2x2 conv's input gradient, NHWC in and out."""
    d = torch.tensor(np.ascontiguousarray(np.transpose(dz_nhwc, (0, 3, 1, 2))), dtype=torch.float64, device=dev)
    y = torch.nn.functional.conv_transpose2d(d, torch.tensor(w, dtype=torch.float64, device=dev))
    return y.permute(0, 2, 3, 1).cpu().numpy()


@pytest.mark.parametrize("ws_dma", ["0", "1", "2"])
@pytest.mark.parametrize("prec", ["f32split", "bf16"])
@pytest.mark.parametrize("shape", [(100, 40, 35, 512), (101, 40, 10, 256), (32, 13, 10, 333)])
def test_conv_forward_tiles_match_own_inputs(shape, prec, ws_dma, monkeypatch):
    """ws_dma: ABD_WS_DMA (read at each launch) -- 0 the direct-load weight-stationary kernels
    everywhere, 1 (default) the LDS-DMA kernel for the forward GEMMs, 2 for the data gradients too."""
    monkeypatch.setenv("ABD_WS_DMA", ws_dma)
    assert torch.cuda.is_available()
    abd_amd.load_library()
    dev = torch.device("cuda", 0)
    H, W, K, B = shape
    g = oc.geometry(H, W)
    lf = g["flat"]
    st = make_state(H, W, K, lf, seed=4100 + H + W + K)
    m = M.smallcnn(K, lf)
    m.load_state_dict({k: torch.tensor(v) for k, v in st.items()})
    m = m.to(dev).train().set_gemm_precision(prec)
    r = np.random.Generator(np.random.PCG64(H * W + B + 11))
    x = torch.tensor(mfcc_like(r, B, H, W), device=dev)
    y = torch.tensor(r.integers(0, K, B), dtype=torch.int64, device=dev)
    eng = m.engine(x)
    m1 = torch.ones((B, lf), dtype=torch.uint8, device=dev)
    m2 = torch.ones((B, 128), dtype=torch.uint8, device=dev)
    ws = eng.workspace(B)
    outs = []
    for _ in range(3):   # do_update=False: the same step three times
        T.train_step(m, x, y, None, None, None, m1, m2, do_update=False, seed=5)
        torch.cuda.synchronize()
        outs.append((ws_array(eng, ws, B, "r2", (B, g["H2"], g["W2"], 64)).copy(),
                     ws_array(eng, ws, B, "r3", (B, g["H3"], g["W3"], 32)).copy(),
                     ws_array(eng, ws, B, "dp1", (B, g["H1p"], g["W1p"], 64)).copy(),
                     ws_array(eng, ws, B, "dp2", (B, g["H2p"], g["W2p"], 64)).copy()))
    for k in (1, 2):
        for a, b in zip(outs[0], outs[k]):
            assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), "conv forward not deterministic"
    r2, r3, dp1, dp2 = (o.astype(np.float64) for o in outs[0])
    rnd = bf16_round if prec == "bf16" else (lambda a: np.asarray(a, np.float64))
    # conv3 from the device's own p2 (BN2 + pool2 output, NHWC)
    p2 = ws_array(eng, ws, B, "p2", (B, g["H2p"], g["W2p"], 64))
    e3 = conv_relu(rnd(p2), rnd(st["conv3.weight"]), st["conv3.bias"].astype(np.float64), dev)
    # conv2 from p1: under the BN1 fold p1 holds m and conv2 applies alpha into its weights and
    # beta' into its bias (the weight side is rounded once to fp32, w * alpha)
    folded = L.lib().abd_smallcnn_bn1_folded(eng.h, B) == 1
    p1 = ws_float(eng, ws, B, "p1", (B, g["H1p"], g["W1p"], 64))
    w2 = st["conv2.weight"].astype(np.float64)
    b2 = st["conv2.bias"].astype(np.float64)
    if folded:
        coef = ws_array(eng, ws, B, "coef", (3, 64, 4))[0].astype(np.float64)
        b2 = b2 + np.einsum("oikl,i->o", w2, coef[:, 3])
        w2 = (st["conv2.weight"] * coef[:, 2].astype(np.float32)[None, :, None, None]).astype(np.float32)
    e2 = conv_relu(rnd(p1), rnd(w2), b2, dev)
    # the data gradients (conv_ws_*_kernel<EPI_STORE>): dp2 = conv3^T dz3, dp1 = conv2^T dz2 from the
    # device's own dz3 / dz2 (dz2 as bf16 planes in bf16's plane mode)
    dz3 = ws_array(eng, ws, B, "dz3", (B, g["H3"], g["W3"], 32))
    dz2 = ws_float(eng, ws, B, "dz2", (B, g["H2"], g["W2"], 64))
    ed2 = conv_t(rnd(dz3), rnd(st["conv3.weight"]), dev)
    ed1 = conv_t(rnd(dz2), rnd(st["conv2.weight"]), dev)
    tol = 1e-5  # fp32 accumulation over K = 256 against the per-utterance max
    for name, got, exp in (("r2", r2, e2), ("r3", r3, e3), ("dp1", dp1, ed1), ("dp2", dp2, ed2)):
        scale = np.abs(exp).max(axis=(1, 2, 3), keepdims=True) + 1e-30
        err = np.abs(got - exp) / scale
        bad = np.argwhere(err > tol)
        assert bad.size == 0, (name, prec, shape, float(err.max()), bad[:5].tolist())
