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
import convergence_stats as CS
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


def _dropin_bddataset():
    """The drop-in prepare_dataset.BDDataset (what the unchanged scripts build, badnets.py:103-104):
    its loaders take training.train()'s HBM-resident fast path (resident.py)."""
    import importlib.util
    import os
    import sys
    if "prepare_dataset" in sys.modules:
        return sys.modules["prepare_dataset"].BDDataset
    d = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "audio-backdoor-attack_amd",
                     "dropin")
    sys.path.insert(0, d)   # for its `import _root`
    try:
        spec = importlib.util.spec_from_file_location("prepare_dataset", os.path.join(d, "prepare_dataset.py"))
        mod = importlib.util.module_from_spec(spec)
        sys.modules["prepare_dataset"] = mod
        spec.loader.exec_module(mod)
    finally:
        sys.path.remove(d)
    return mod.BDDataset


def fix_random(seed=35):
    """utils/random_tools.py:5-18"""
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    torch.cuda.manual_seed_all(seed)


_DATA = {}


def eval_model(name, dev, source, ref, prec="f32", rng_seed=None):
    """One eval_model run (badnets.py:127-160).  rng_seed: re-seed torch (CPU batch orders, device
    dropout) after the data are built -- another draw of the run, as make_convergence.py's
    SEED_REPLICATES do for the reference."""
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
    if rng_seed is not None:
        torch.manual_seed(rng_seed)
    B = c["B"]
    BDDataset = _dropin_bddataset()
    clean = torch.utils.data.DataLoader(torch.utils.data.TensorDataset(torch.tensor(d["clean_x"]),
                                                                       torch.tensor(d["clean_y"])),
                                        batch_size=B, shuffle=True)
    bd_train = torch.utils.data.DataLoader(BDDataset(torch.tensor(d["bd_x"]), torch.tensor(d["bd_y"]),
                                                     torch.tensor(d["ind"])), batch_size=B, shuffle=True)
    bd_test = torch.utils.data.DataLoader(BDDataset(torch.tensor(d["bt_x"]), torch.tensor(d["bt_y"]),
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


# ---------------------------------------------------------------------------------------------
# Per-epoch clean accuracy / ASR against the reference's run-to-run distribution.
# A device-dropout run (and a bf16 run: its rounded operands move the trajectory off the reference's
# within a few epochs) is another DRAW of the attack, not a replay: other masks, other batch orders.
# make_convergence.py ran the reference's loop under further torch seeds on the same init and data
# (<name>_test_seeds_ep / _train_seeds_ep); with the fixture run itself that is R reference draws
# per epoch.  D device runs (other seeds) are averaged and compared at EVERY epoch, for test clean
# accuracy, test ASR, train accuracy and train ASR, with convergence_stats.draw_bound (K sigma of
# the difference of the two means).  Many epoch-metric cells are compared per test, so the test
# allows at most CS.MAX_CELLS (2) cells past the bound and none past CS.MAX_RATIO (2x) it --
# calibrated on the reference's draws alone (leave-D-out: D of them in place of the device runs, the rest as the reference, every
# split; tests/test_convergence_calibration_cpu.py).
# Device draws per config: 8, and 48 for FlowMur, whose clean-label ASR is the noisiest metric
# (sd up to 6.5 pp per draw; the reference side has 41 draws of it, make_convergence.py
# SEED_REPLICATES, and its K is 3.5: convergence_stats.K_BY_CFG) -- so its test-ASR bound is <= 5 pp at
# every epoch and a 4-5 pp shift is caught (test_convergence_calibration_cpu.py).
D_RUNS = {"flowmur": 48}
D_DEFAULT = 8
DEV_SEEDS = (None,) + tuple(range(2001, 2060))


def n_draws(name):
    return D_RUNS.get(name, D_DEFAULT)


def check_draws(name, label, runs, conv_ref, d):
    """runs: list of (tr, te) arrays of the device draws; asserts every epoch and metric."""
    c = CONV_CFGS[name]
    dens = {"n_test": c["n_test"], "n_train": c["n_train"], "n_bd": int(d["bt_ind"].sum()),
            "n_pois": int(d["ind"].sum())}
    rte, rtr = CS.ref_draws(conv_ref, name)
    ote, otr = np.stack([te for _, te in runs]), np.stack([tr for tr, _ in runs])
    refs, ours = {"te": rte, "tr": rtr}, {"te": ote, "tr": otr}
    unsat = 0
    print(f"\n{name} [{label}]: per epoch, mean of {len(runs)} draw(s) vs the reference's {rte.shape[0]} draws "
          "(mean +- sd) and the allowed gap")
    for what, src, col, den in CS.METRICS:
        r, o = refs[src][:, :, col], ours[src][:, :, col]
        bound = CS.draw_bound(r, o.shape[0], dens[den])
        gap = np.abs(o.mean(0) - r.mean(0))
        print(f"  {what}:")
        for e in range(r.shape[1]):
            unsat += int(r[:, e].mean() < 99.0)
            flag = "" if gap[e] <= bound[e] else "  <-- outside"
            print(f"    epoch {e + 1:2d}: ours {o[:, e].mean():7.3f}  ref {r[:, e].mean():7.3f} +- {r[:, e].std(ddof=1):6.3f}"
                  f"  gap {gap[e]:6.3f} <= {bound[e]:6.3f}{flag}")
    assert unsat > 0, "no unsaturated epoch compared"
    bad = CS.violations(ote, otr, rte, rtr, dens, k_sigma=CS.k_sigma(name, len(runs)))
    assert not CS.rule_fails(bad), bad
    # final epoch: the mean of the draws' final clean accuracy / ASR against the
    # reference's own final, within final_allowed's device bound -- max(0.5 pp, the reference's
    # implementation spread, the range of its own RNG replicates)
    for col, what in ((0, "clean acc"), (1, "ASR")):
        allowed = final_allowed(conv_ref, name, col, "device")
        got, ref = float(ote[:, -1, col].mean()), float(conv_ref[f"{name}_test"][-1, col])
        print(f"  final {what}: mean of draws {got:.3f} vs reference {ref:.3f} (allowed {allowed:.3f})")
        assert abs(got - ref) <= allowed, (what, got, ref, allowed)


@pytest.mark.parametrize("prec", ["f32", "f32split"])
@pytest.mark.parametrize("name", list(CONV_CFGS))
def test_device_dropout_epochs_within_reference_draws(dev, conv_ref, name, prec):
    runs = []
    for sd in DEV_SEEDS[:n_draws(name)]:
        tr, te, _, d = eval_model(name, dev, "device", conv_ref, prec, rng_seed=sd)
        assert tr[-1, 0] < tr[0, 0]                              # training converges
        runs.append((tr, te))
    check_draws(name, f"{prec}, device dropout", runs, conv_ref, d)


# bf16 conv GEMMs (BASELINE configs[2] jingleback and configs[4] flowmur name bf16; badnets shares
# jingleback's 101 x 40 geometry): per-epoch losses are not expected to track the fp32 reference
# at 1e-4 (operands rounded to 8 significand bits), so both dropout modes are held to the
# reference's draw distribution at every epoch (check_draws); the replay with the reference's own
# masks also prints its gap to the fp32 replay bound (max(0.5 pp, 3x the reference's
# implementation spread) at that epoch) for DESIGN.md §4.
BF16_CFGS = [n for n in ("badnets", "jingleback", "flowmur") if n in CONV_CFGS]
# The bf16 replay is held to the fp32 replay bound at every epoch.  FlowMur's misses it (round 5:
# epoch 1 clean accuracy 0.68 pp against 0.50, epoch 4 ASR 2.56 pp against 0.64; its clean-label ASR
# moves between the reference's own fp32 implementations too): an OPEN known
# limitation, tracked as a non-strict xfail so the suite reports it every run (XPASS if it closes),
# beside the draw bound it does meet.
BF16_REPLAY_OPEN = ("flowmur",)


@pytest.mark.parametrize("name", [pytest.param(n, marks=pytest.mark.xfail(
    reason="known limitation: FlowMur bf16 replay past the fp32 replay bound (DESIGN.md §4)", strict=False))
    if n in BF16_REPLAY_OPEN else n for n in BF16_CFGS])
def test_bf16_replay_fp32_bound(dev, conv_ref, name):
    """bf16 with the reference's own masks: clean accuracy / ASR within the fp32 replay bound
    (max(0.5 pp, 3x the reference's implementation spread, two samples)) at EVERY epoch."""
    tr, te, _, d = eval_model(name, dev, "torch_cpu", conv_ref, "bf16")
    rte, s_te = conv_ref[f"{name}_test"], conv_ref[f"{name}_test_alt"]
    n_bd = int(d["bt_ind"].sum())
    tight = []
    for e in range(len(rte)):
        b_acc = max(0.5, 3.0 * abs(s_te[e, 0] - rte[e, 0]), 200.0 / CONV_CFGS[name]["n_test"])
        b_asr = max(0.5, 3.0 * abs(s_te[e, 1] - rte[e, 1]), 200.0 / n_bd)
        if abs(te[e, 0] - rte[e, 0]) > b_acc + 1e-6 or abs(te[e, 1] - rte[e, 1]) > b_asr + 1e-6:  # <= (counts)
            tight.append((e + 1, round(abs(te[e, 0] - rte[e, 0]), 3), round(b_acc, 3),
                          round(abs(te[e, 1] - rte[e, 1]), 3), round(b_asr, 3)))
    assert not tight, ("bf16 replay past the fp32 replay bound (epoch, acc gap, bound, ASR gap, bound)", tight)


@pytest.mark.parametrize("name", BF16_CFGS)
def test_bf16_replay_epochs(dev, conv_ref, name):
    tr, te, _, d = eval_model(name, dev, "torch_cpu", conv_ref, "bf16")
    rtr, rte = conv_ref[f"{name}_train"], conv_ref[f"{name}_test"]
    s_te = conv_ref[f"{name}_test_alt"]
    rel = lambda a, b: np.abs(a - b) / np.maximum(np.abs(b), 1e-12)  # noqa: E731
    n_bd = int(d["bt_ind"].sum())
    print(f"\n{name} [bf16, reference masks] per epoch: |train loss - ref| / ref; clean acc / ASR GPU vs "
          "reference, and the fp32 replay bound")
    tight = []
    for e in range(len(rtr)):
        b_acc = max(0.5, 3.0 * abs(s_te[e, 0] - rte[e, 0]), 200.0 / CONV_CFGS[name]["n_test"])
        b_asr = max(0.5, 3.0 * abs(s_te[e, 1] - rte[e, 1]), 200.0 / n_bd)
        print(f"  epoch {e + 1:2d}: {rel(tr[e, 0], rtr[e, 0]):.1e}  {te[e, 0]:7.3f}/{te[e, 1]:7.3f} vs "
              f"{rte[e, 0]:7.3f}/{rte[e, 1]:7.3f}  gaps {abs(te[e, 0] - rte[e, 0]):6.3f} (<= {b_acc:.3f}?) "
              f"{abs(te[e, 1] - rte[e, 1]):6.3f} (<= {b_asr:.3f}?)")
        if abs(te[e, 0] - rte[e, 0]) > b_acc + 1e-6 or abs(te[e, 1] - rte[e, 1]) > b_asr + 1e-6:  # <= (counts)
            tight.append(e + 1)
    print(f"  epochs past the fp32 replay bound: {tight} (test_bf16_replay_fp32_bound)")
    assert tr[-1, 0] < tr[0, 0]
    check_draws(name, "bf16, reference masks", [(tr, te)], conv_ref, d)


@pytest.mark.parametrize("name", BF16_CFGS)
def test_bf16_device_dropout_epochs_within_reference_draws(dev, conv_ref, name):
    runs = []
    for sd in DEV_SEEDS[:n_draws(name)]:
        tr, te, _, d = eval_model(name, dev, "device", conv_ref, "bf16", rng_seed=sd)
        assert tr[-1, 0] < tr[0, 0]
        runs.append((tr, te))
    check_draws(name, "bf16, device dropout", runs, conv_ref, d)
