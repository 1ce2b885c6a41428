"""GPU: the bf16-MFMA conv GEMMs (abd_smallcnn_set_precision / smallcnn.set_gemm_precision):
opt-in 'bf16' and the fp32-accurate 'f32split' (three exact bf16 planes per operand, six terms).

Kernel exactness: each bf16 GEMM output the device wrote (conv2/conv3 forward -> r2/r3,
conv3/conv2 data gradients -> dp2/dp1) equals the float64 product of the SAME device inputs
rounded to bf16 (RNE) -- only the fp32 accumulation order differs.  Model level: bf16 log-probs
stay within bf16 tolerance of the fp32 path, and training on a separable synthetic task tracks
the fp32 loss curve.
"""
import numpy as np
import pytest
import torch

import abd_amd
from abd_amd import models as M, training as T, _lib as L
from golden_inputs import make_state, mfcc_like
from oracle import smallcnn as oc
from gpu_replay import ws_float

pytestmark = pytest.mark.gpu


def bf16(a):
    """float32 -> bf16 (round to nearest even) -> float64."""
    u = np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)
    r = ((u >> 16) & 1) + np.uint32(0x7FFF)
    return ((u + r) & np.uint32(0xFFFF0000)).view(np.float32).astype(np.float64)


def ws_view(eng, ws, B, name, shape):
    off = L.lib().abd_smallcnn_workspace_offset(eng.h, B, name.encode())
    assert off >= 0, name
    n = int(np.prod(shape)) * 4
    return ws[off:off + n].view(torch.float32).view(*shape).cpu().numpy().astype(np.float64)


def nchw(a):
    return np.transpose(a, (0, 3, 1, 2))


def nrel(a, b):
    return float(np.linalg.norm(np.asarray(a) - np.asarray(b)) / max(np.linalg.norm(b), 1e-30))


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    abd_amd.load_library()
    return torch.device("cuda", 0)


@pytest.mark.parametrize("prec", ["bf16", "f32split"])
@pytest.mark.parametrize("shape", [(101, 40, 10, 64), (32, 13, 10, 40)])
def test_bf16_gemms_exact_on_rounded_operands(dev, shape, prec):
    """bf16: exact products of the bf16-rounded operands.  f32split: the six-term exact bf16
    split of the UNROUNDED fp32 operands -- the same 2e-6 bound as against the float64 product."""
    H, W, K, B = shape
    rnd = bf16 if prec == "bf16" else (lambda a: np.asarray(a, np.float64))
    g = oc.geometry(H, W)
    st = make_state(H, W, K, g["flat"], seed=77 + H)
    m = M.smallcnn(K, g["flat"])
    m.load_state_dict({k: torch.tensor(v) for k, v in st.items()})
    m = m.to(dev).train().set_gemm_precision(prec)
    r = np.random.Generator(np.random.PCG64(H + B))
    x = torch.tensor(mfcc_like(r, B, H, W), device=dev)
    y = torch.tensor(r.integers(0, K, B), device=dev)
    eng = m.engine(x)
    T.train_step(m, x, y, torch.zeros(B, dtype=torch.int64, device=dev), None, None, seed=3)
    torch.cuda.synchronize()
    ws = eng.workspace(B)
    p1 = ws_float(eng, ws, B, "p1", (B, g["H1p"], g["W1p"], 64))   # fp32 buffer or conv2 planes
    r2 = ws_view(eng, ws, B, "r2", (B, g["H2"], g["W2"], 64))
    p2 = ws_view(eng, ws, B, "p2", (B, g["H2p"], g["W2p"], 64))
    r3 = ws_view(eng, ws, B, "r3", (B, g["H3"], g["W3"], 32))
    dz3 = ws_view(eng, ws, B, "dz3", (B, g["H3"], g["W3"], 32))
    dp2 = ws_view(eng, ws, B, "dp2", (B, g["H2p"], g["W2p"], 64))
    dz2 = ws_float(eng, ws, B, "dz2", (B, g["H2"], g["W2"], 64))
    dp1 = ws_view(eng, ws, B, "dp1", (B, g["H1p"], g["W1p"], 64))
    w2 = rnd(st["conv2.weight"])
    w3 = rnd(st["conv3.weight"])
    b2 = st["conv2.bias"].astype(np.float64)
    folded = L.lib().abd_smallcnn_bn1_folded(eng.h, B) == 1
    p1_true, w2f = p1, w2
    if folded:
        # f32split train step: p1 holds m; conv2 runs on fl32(w * alpha_c) and bias b + sum w beta'_c
        # (conv1_stats_fold_kernel / conv_ws_split_kernel fold): the GEMM is checked on those operands
        c1 = ws_view(eng, ws, B, "coef", (3, 64, 4))[0]
        w2f = rnd((st["conv2.weight"].astype(np.float32) * c1[None, :, None, None, 2].astype(np.float32)))
        b2 = (b2 + np.einsum("ncij,c->n", st["conv2.weight"].astype(np.float64), c1[:, 3])).astype(np.float32)
        p1_true = p1 * c1[:, 2] + c1[:, 3]
    ref_r2 = np.maximum(oc.conv2x2(rnd(nchw(p1)), w2f, b2.astype(np.float64)), 0.0)
    ref_r3 = np.maximum(oc.conv2x2(rnd(nchw(p2)), w3, st["conv3.bias"].astype(np.float64)), 0.0)
    ref_dp2, _, _ = oc.conv2x2_backward(np.zeros((B, 64, g["H2p"], g["W2p"])), w3, rnd(nchw(dz3)))
    ref_dp1, _, _ = oc.conv2x2_backward(np.zeros((B, 64, g["H1p"], g["W1p"])), w2, rnd(nchw(dz2)))
    errs = {"r2": nrel(nchw(r2), ref_r2), "r3": nrel(nchw(r3), ref_r3), "dp2": nrel(nchw(dp2), ref_dp2),
            "dp1": nrel(nchw(dp1), ref_dp1)}
    # weight gradients (conv_wgrad_trp_kernel: six split terms / one bf16 term): the products of the
    # same device operands, rounded; under the fold conv2's is taken over m and unfolded
    # (alpha_c G_m + beta'_c db_n, slab_reduce_kernel)
    grads = {n: v.cpu().numpy().astype(np.float64) for n, v in zip(M.PARAM_ORDER, eng.views(eng.grads))}
    _, gw3, _ = oc.conv2x2_backward(rnd(nchw(p2)), w3, rnd(nchw(dz3)))
    _, gw2, _ = oc.conv2x2_backward(rnd(nchw(p1)), w2, rnd(nchw(dz2)))
    if folded:
        gw2 = gw2 * c1[None, :, None, None, 2] + c1[None, :, None, None, 3] * grads["conv2.bias"][:, None, None, None]
    wg = {"conv3.weight": nrel(grads["conv3.weight"].reshape(gw3.shape), gw3),
          "conv2.weight": nrel(grads["conv2.weight"].reshape(gw2.shape), gw2)}
    print(shape, prec, "folded" if folded else "", {k: f"{v:.1e}" for k, v in {**errs, **wg}.items()})
    for k, v in errs.items():
        assert v < 2e-6, (k, v)
    for k, v in wg.items():
        assert v < 1e-5, (k, v)
    # and the products really are bf16: the exact-fp32 product differs by ~bf16 rounding
    ref32 = np.maximum(oc.conv2x2(nchw(p1_true), st["conv2.weight"].astype(np.float64),
                                  st["conv2.bias"].astype(np.float64)), 0.0)
    if prec == "bf16":
        assert nrel(nchw(r2), ref32) > 1e-4
    else:  # folded: against the unfolded layer, within the fold's one extra rounding per weight
        assert nrel(nchw(r2), ref32) < (1e-5 if folded else 2e-6)


def test_bf16_logprobs_close_to_fp32(dev):
    H, W, K, B = 100, 40, 35, 128
    g = oc.geometry(H, W)
    st = make_state(H, W, K, g["flat"], seed=5, trained_bn=True)
    out = {}
    for prec in ("f32", "bf16"):
        m = M.smallcnn(K, g["flat"])
        m.load_state_dict({k: torch.tensor(v) for k, v in st.items()})
        m = m.to(dev).eval().set_gemm_precision(prec)
        x = torch.tensor(mfcc_like(np.random.Generator(np.random.PCG64(9)), B, H, W), device=dev)
        with torch.no_grad():
            out[prec] = m(x).cpu().numpy().astype(np.float64)
    err = nrel(out["bf16"], out["f32"])
    agree = np.mean(out["bf16"].argmax(1) == out["f32"].argmax(1))
    print("bf16 vs f32 log-probs", err, "argmax agreement", agree)
    assert 1e-6 < err < 2e-2 and agree > 0.95


def test_bf16_training_tracks_fp32(dev):
    from abd_amd import synth
    from abd_amd.pipeline import ResidentTrainer, attack_config
    cfg = attack_config("badnets")
    waves, labels = synth.make_clips_torch(1024, 16000, 16000, 10, seed=11, device=dev)
    res = {}
    for prec in ("f32", "bf16"):
        torch.manual_seed(35)
        m = M.smallcnn(10, 3072).to(dev)
        opt = torch.optim.Adam(m.parameters(), lr=1e-3)
        tr = ResidentTrainer(cfg, waves, labels, m, opt, 128, seed=35, gemm_precision=prec)
        hist = [tr.run_epoch()["loss"] for _ in range(3)]
        res[prec] = hist
    print(res)
    assert res["bf16"][-1] < res["bf16"][0]                      # it learns
    assert abs(res["bf16"][-1] - res["f32"][-1]) < 0.15 * res["f32"][0]
