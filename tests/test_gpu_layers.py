"""GPU: layer-by-layer comparison of every smallcnn activation / gradient buffer with the oracle."""
import ctypes as C

import numpy as np
import pytest
import torch

import abd_amd
from abd_amd import models as M, training as T, _lib as L
from golden_inputs import make_state, mfcc_like, patch
from oracle import smallcnn as oc
from gpu_replay import decisions, ws_float

pytestmark = pytest.mark.gpu


def nrel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def ws_view(eng, ws, B, name, shape, dtype=torch.float32):
    off = L.lib().abd_smallcnn_workspace_offset(eng.h, B, name.encode())
    assert off >= 0, name
    n = int(np.prod(shape)) * torch.tensor([], dtype=dtype).element_size()
    return ws[off:off + n].view(dtype).view(*shape).cpu().numpy()


@pytest.mark.parametrize("prec", ["f32", "f32split"])
@pytest.mark.parametrize("shape", [(101, 40, 10, 64), (32, 13, 10, 48), (32, 40, 10, 1)])
def test_every_buffer_matches_oracle(shape, prec):
    """prec 'f32split' also covers the train step's BN1 fold into conv2 (conv1_stats_fold_kernel)."""
    assert torch.cuda.is_available()
    abd_amd.load_library()
    dev = torch.device("cuda", 0)
    H, W, K, B = shape
    g = oc.geometry(H, W)
    lf = g["flat"]
    st = make_state(H, W, K, lf, seed=3000 + H + W + K)
    m = M.smallcnn(K, lf)
    m.load_state_dict({k: torch.tensor(v) for k, v in st.items()})
    m = m.to(dev).train().set_gemm_precision(prec)
    r = np.random.Generator(np.random.PCG64(H * W + B))
    x = mfcc_like(r, B, H, W)
    y = r.integers(0, K, B).astype(np.int64)
    ind = (r.random(B) < 0.2).astype(np.int64)
    for i in np.nonzero(ind)[0]:
        patch(x[i:i + 1])
        y[i] = 2
    xd = torch.tensor(x, device=dev)
    eng = m.engine(xd)
    mo = (torch.empty((B, lf), dtype=torch.uint8, device=dev), torch.empty((B, 128), dtype=torch.uint8, device=dev))
    T.train_step(m, xd, torch.tensor(y, device=dev), torch.tensor(ind, device=dev), None, None, masks_out=mo, seed=7)
    torch.cuda.synchronize()
    ws = eng.workspace(B)
    o = oc.SmallCNN(st)
    m1, m2 = mo[0].cpu().numpy(), mo[1].cpu().numpy()
    force = decisions(eng, B, x, st, g)
    out, c = o.forward_train(x, m1, m2, force=force)
    replayed = {i: c[f"replayed{i}"] for i in (1, 2, 3)}
    _, dz = o.ce_loss_and_grad(out, y)
    rec = {}
    o.backward(c, dz, record=rec)
    nhwc = lambda a: np.transpose(a, (0, 2, 3, 1))  # noqa: E731
    checks = [
        ("p1", c["in2"], nhwc, (B, g["H1p"], g["W1p"], 64), 1e-5),
        ("r2", c["r2"], nhwc, (B, g["H2"], g["W2"], 64), 1e-5),
        ("p2", c["in3"], nhwc, (B, g["H2p"], g["W2p"], 64), 1e-5),
        ("r3", c["r3"], nhwc, (B, g["H3"], g["W3"], 32), 1e-5),
        ("p3d", c["d1"], None, (B, lf), 1e-5),
        ("d2", c["d2"], None, (B, 128), 1e-5),
        ("dz", dz, None, (B, K), 1e-5),
        ("da", rec["da"], None, (B, 128), 1e-5),
        ("dp3", rec["dp3"], None, (B, lf), 1e-5),
        ("dz3", rec["dz3"], nhwc, (B, g["H3"], g["W3"], 32), 1e-5),
        ("dp2", rec["dp2"], nhwc, (B, g["H2p"], g["W2p"], 64), 1e-5),
        ("dz2", rec["dz2"], nhwc, (B, g["H2"], g["W2"], 64), 1e-5),
        ("dp1", rec["dp1"], nhwc, (B, g["H1p"], g["W1p"], 64), 1e-5),
    ]
    # f32split train step: BN1 folded into conv2, p1's buffer holds the pool-selected relu(conv1) m
    folded = L.lib().abd_smallcnn_bn1_folded(eng.h, B) == 1
    coef1 = ws_view(eng, ws, B, "coef", (3, 64, 4))[0]
    report = {}
    for name, ref, tf, shp, tol in checks:
        got = ws_float(eng, ws, B, name, shp) if name in ("p1", "dz2") else ws_view(eng, ws, B, name, shp)
        if name == "p1" and folded:  # p1 = alpha * m + beta' (what conv2's folded weights / bias apply)
            got = got.astype(np.float64) * coef1[:, 2] + coef1[:, 3]
        refv = tf(ref) if tf else ref
        report[name] = nrel(got, refv)
    print(shape, prec, "folded" if folded else "", "replayed decisions", replayed, {k: f"{v:.1e}" for k, v in report.items()})
    for name, ref, tf, shp, tol in checks:
        assert report[name] < tol, (name, report[name])
