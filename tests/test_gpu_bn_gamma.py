"""GPU: BatchNorm backward with vanishing gamma.

The train step derives BN1/BN2/BN3's backward statistics from the next layer's gradients; the
unfolded forms read xhat back as (p - beta) / gamma, which is 0/0 at gamma = 0 and amplifies fp32
rounding by |beta| / |gamma| near it.  Under the BN1 fold the derivation is division-free
(invstd * sum W (G_m - mean db)); elsewhere a guarded fallback recomputes the layer's statistics
from the activations when a channel's gamma is tiny.  Every parameter gradient and every
backward buffer is compared with the float64 oracle with gamma in {0, 1e-4, -1e-4} on three
channels of each BatchNorm.
"""
import numpy as np
import pytest
import torch

import abd_amd
from abd_amd import models as M, training as T
from golden_inputs import make_state, mfcc_like
from gpu_replay import decisions, ws_float
from oracle import smallcnn as oc
from test_gpu_layers import ws_view, nrel

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("prec", ["f32", "f32split"])
def test_tiny_gamma_gradients_match_oracle(prec):
    assert torch.cuda.is_available()
    abd_amd.load_library()
    dev = torch.device("cuda", 0)
    H, W, K, B = 101, 40, 10, 64
    g = oc.geometry(H, W)
    lf = g["flat"]
    st = make_state(H, W, K, lf, seed=77)
    for i in (1, 2, 3):
        gm = st[f"bn{i}.weight"].copy()
        gm[:3] = [0.0, 1e-4, -1e-4]
        st[f"bn{i}.weight"] = gm
        bt = st[f"bn{i}.bias"].copy()
        bt[:3] = [0.7, -0.4, 0.25]
        st[f"bn{i}.bias"] = bt
    m = M.smallcnn(K, lf)
    m.load_state_dict({k: torch.tensor(v) for k, v in st.items()})
    m = m.to(dev).train().set_gemm_precision(prec)
    r = np.random.Generator(np.random.PCG64(1234))
    x = mfcc_like(r, B, H, W)
    y = r.integers(0, K, B).astype(np.int64)
    xd = torch.tensor(x, device=dev)
    eng = m.engine(xd)
    mo = (torch.empty((B, lf), dtype=torch.uint8, device=dev), torch.empty((B, 128), dtype=torch.uint8, device=dev))
    T.train_step(m, xd, torch.tensor(y, device=dev), None, None, None, masks_out=mo, seed=7)
    torch.cuda.synchronize()
    grads = {n: v.view(p.shape).cpu().numpy() for n, v, p in
             zip(M.PARAM_ORDER, eng.views(eng.grads), m._param_list())}
    assert all(np.isfinite(v).all() for v in grads.values()), [n for n, v in grads.items() if not np.isfinite(v).all()]
    o = oc.SmallCNN(st)
    force = decisions(eng, B, x, st, g)
    out, c = o.forward_train(x, mo[0].cpu().numpy(), mo[1].cpu().numpy(), force=force)
    _, dz = o.ce_loss_and_grad(out, y)
    rec = {}
    ref = o.backward(c, dz, record=rec)
    report = {n: nrel(grads[n], ref[n]) for n in M.PARAM_ORDER}
    nhwc = lambda a: np.transpose(a, (0, 2, 3, 1))  # noqa: E731
    ws = eng.workspace(B)
    for name, shp in (("dz3", (B, g["H3"], g["W3"], 32)), ("dz2", (B, g["H2"], g["W2"], 64))):
        report[name] = nrel(ws_float(eng, ws, B, name, shp), nhwc(rec[name]))
    # the tiny channels' own BN gradients, elementwise against the layer's scale
    for i in (1, 2, 3):
        for n in (f"bn{i}.weight", f"bn{i}.bias"):
            scale = np.abs(ref[n]).max()
            report[n + "[:3]"] = float(np.abs(grads[n][:3] - ref[n][:3]).max() / scale)
    print(prec, {k: f"{v:.1e}" for k, v in report.items()})
    bad = {k: v for k, v in report.items() if not v < 1e-4}
    assert not bad, bad
