"""The BatchNorm backward statistics the HIP path derives from the next conv's gradients.

libabd forms BN1's and BN2's backward sums (sum dy, sum dy * xhat) without a pass over the
activations (csrc/smallcnn.hip ``bn_bwd_derived_kernel``): max-pool routes each pooled gradient
dp to one element whose normalised value is (p - beta) / gamma, and dp = conv^T(dz), so

    sum dy        = sum_{n,t} W[n,c,t] * db[n]
    sum dy * xhat = sum_{n,t} W[n,c,t] * (G[n,c,t] - beta_c * db[n]) / gamma_c

with G, db the conv's weight and bias gradients.  This checks the identity on the float64
oracle (utils/models.py:17-65 restated in oracle/smallcnn.py) for random parameters,
including negative gammas (pooling then selects the minimum of the pre-BN activations).
"""
import numpy as np
import pytest

from oracle import smallcnn as oc


def _state(rng, H0, W0, K):
    g = oc.geometry(H0, W0)
    shapes = {
        "conv1.weight": (64, 1, 2, 2), "conv1.bias": (64,), "bn1.weight": (64,), "bn1.bias": (64,),
        "conv2.weight": (64, 64, 2, 2), "conv2.bias": (64,), "bn2.weight": (64,), "bn2.bias": (64,),
        "conv3.weight": (32, 64, 2, 2), "conv3.bias": (32,), "bn3.weight": (32,), "bn3.bias": (32,),
        "fc1.weight": (128, g["flat"]), "fc1.bias": (128,), "fc2.weight": (K, 128), "fc2.bias": (K,),
    }
    st = {k: rng.standard_normal(s) * 0.3 for k, s in shapes.items()}
    for i in (1, 2, 3):
        gam = rng.uniform(0.5, 1.5, st[f"bn{i}.weight"].shape)
        gam[::5] *= -1.0  # negative gammas: pool picks the BN output's max = pre-BN min
        st[f"bn{i}.weight"] = gam
        st[f"bn{i}.bias"] = rng.standard_normal(gam.shape) * 0.5
    for i in (1, 2, 3):
        C = 64 if i < 3 else 32
        st[f"bn{i}.running_mean"] = np.zeros(C)
        st[f"bn{i}.running_var"] = np.ones(C)
    return st, g


@pytest.mark.parametrize("H0,W0,K", [(20, 40, 10), (17, 12, 5)])
def test_bn_backward_sums_from_conv_gradients(H0, W0, K):
    rng = np.random.default_rng(7)
    st, g = _state(rng, H0, W0, K)
    m = oc.SmallCNN(st, K)
    B = 6
    x = rng.standard_normal((B, 1, H0, W0))
    m1 = (rng.random((B, g["flat"])) > 0.4).astype(np.float64)
    m2 = (rng.random((B, 128)) > 0.5).astype(np.float64)
    out, c = m.forward_train(x, m1, m2)
    labels = rng.integers(0, K, B)
    _, dz = m.ce_loss_and_grad(out, labels)
    rec = {}
    grads = m.backward(c, dz, record=rec)
    for i, nxt in ((1, 2), (2, 3)):
        W = m.p[f"conv{nxt}.weight"]
        Gw, db = grads[f"conv{nxt}.weight"], grads[f"conv{nxt}.bias"]
        beta, gamma = m.p[f"bn{i}.bias"], m.p[f"bn{i}.weight"]
        sdy = np.einsum("nct,n->c", W.reshape(W.shape[0], W.shape[1], 4), db)
        sdyx = np.einsum("nct,nct->c", W.reshape(W.shape[0], W.shape[1], 4),
                         Gw.reshape(W.shape[0], W.shape[1], 4) - beta[None, :, None] * db[:, None, None]) / gamma
        # direct: the BN weight / bias gradients are exactly these sums (oracle bn_backward)
        np.testing.assert_allclose(sdy, grads[f"bn{i}.bias"], rtol=1e-9, atol=1e-12)
        np.testing.assert_allclose(sdyx, grads[f"bn{i}.weight"], rtol=1e-9, atol=1e-12)


@pytest.mark.parametrize("H0,W0,K", [(20, 40, 10), (17, 12, 5)])
def test_bn1_fold_identities(H0, W0, K):
    """The train step's BN1 fold (csrc/smallcnn.hip conv1_stats_fold_kernel, conv_ws_split_kernel
    fold, unfold_wgrad): pool1 of BN1's output equals alpha * m + beta' with m the window's max
    relu(conv1) for gamma >= 0 and its min for gamma < 0; conv2 over m with w * alpha and
    b + sum w * beta' equals conv2 over p1; the weight gradient over m unfolds to the one over p1."""
    rng = np.random.default_rng(11)
    st, g = _state(rng, H0, W0, K)
    m = oc.SmallCNN(st, K)
    B = 5
    x = rng.standard_normal((B, 1, H0, W0))
    out, c = m.forward_train(x, np.ones((B, g["flat"])), np.ones((B, 128)))
    r1, bn = c["r1"], c["bn1"]
    gam, bet = m.p["bn1.weight"], m.p["bn1.bias"]
    alpha = gam * bn["invstd"]
    betap = bet - bn["mean"] * alpha
    W1p = g["W1p"]
    win = r1[:, :, :, :3 * W1p].reshape(B, 64, g["H1"], W1p, 3)
    msel = np.where((gam < 0)[None, :, None, None], win.min(-1), win.max(-1))
    p1 = alpha[None, :, None, None] * msel + betap[None, :, None, None]
    np.testing.assert_allclose(p1, c["in2"], rtol=1e-12, atol=1e-12)
    W2, b2 = m.p["conv2.weight"], m.p["conv2.bias"]
    wf = W2 * alpha[None, :, None, None]
    bf = b2 + np.einsum("ncij,c->n", W2, betap)
    np.testing.assert_allclose(oc.conv2x2(msel, wf, bf), oc.conv2x2(c["in2"], W2, b2), rtol=1e-10, atol=1e-10)
    dz = rng.standard_normal((B, 64, g["H2"], g["W2"]))
    _, gm, db = oc.conv2x2_backward(msel, W2, dz, need_dx=False)
    _, gp, _ = oc.conv2x2_backward(c["in2"], W2, dz, need_dx=False)
    unf = alpha[None, :, None, None] * gm + betap[None, :, None, None] * db[:, None, None, None]
    np.testing.assert_allclose(unf, gp, rtol=1e-10, atol=1e-10)
