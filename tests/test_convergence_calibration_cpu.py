"""CPU: the false-alarm rate AND the power of the per-epoch draw check, measured on the reference's own draws.

tests/test_gpu_convergence.py holds D device-dropout (or bf16) runs to the reference's R draws at
every epoch (convergence_stats.draw_bound) and allows at most MAX_CELLS epoch-metric cells past the
bound, none past MAX_RATIO times it.  Here leave-D-out splits of the reference's draws play both
roles -- D of them as "device" runs, the other R - D as the reference -- so the rule's false-alarm
rate on runs that ARE the reference's distribution is measured, not assumed: every split for the
9-draw configs (D = 3), 2,000 seeded random splits for FlowMur's 41 draws (D = 16).  The bound
normalises by sd * sqrt(1/D + 1/R), so these (D, R) stand for the GPU test's (8 or 48, all R).

Power: the same splits with the "device" draws shifted down by a systematic amount on
one metric must fail the rule; and convergence_stats.detectable_shift gives, for the GPU test's own
(D, R), the smallest shift the rule catches in 90 % of runs (DESIGN.md §4 lists them)."""
import itertools

import numpy as np
import pytest

import convergence_stats as CS
from golden_inputs import CONV_CFGS

D_CAL = {"flowmur": 16}
N_RANDOM = 2000
GPU_D = {"flowmur": 48}   # tests/test_gpu_convergence.py D_RUNS / D_DEFAULT
GPU_D_DEFAULT = 8


@pytest.fixture(scope="module")
def conv_ref():
    import os
    p = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "convergence_ref.npz")
    return dict(np.load(p))


def _dens(name):
    c = CONV_CFGS[name]
    return {"n_test": c["n_test"], "n_train": c["n_train"], "n_bd": 0.9 * c["n_test"], "n_pois": 0.1 * c["n_train"]}


def _splits(name, R):
    D = D_CAL.get(name, 3)
    if D == 3:
        return D, list(itertools.combinations(range(R), D))
    rng = np.random.default_rng(35)
    return D, [tuple(sorted(rng.choice(R, size=D, replace=False))) for _ in range(N_RANDOM)]


def test_gpu_test_draw_counts_match():
    import test_gpu_convergence as G
    for name in CONV_CFGS:
        assert G.n_draws(name) == GPU_D.get(name, GPU_D_DEFAULT), name


@pytest.mark.parametrize("name", list(CONV_CFGS))
def test_draw_rule_false_alarm_rate(conv_ref, name):
    te, tr = CS.ref_draws(conv_ref, name)
    R = te.shape[0]
    assert R >= 9, R
    dens, k = _dens(name), CS.k_sigma(name)
    D, splits = _splits(name, R)
    fails, cells = 0, 0
    for dev in splits:
        rest = [i for i in range(R) if i not in dev]
        bad = CS.violations(te[list(dev)], tr[list(dev)], te[rest], tr[rest], dens, k_sigma=k)
        cells += len(bad)
        fails += int(CS.rule_fails(bad))
    print(f"{name}: K {k}, D {D} of R {R}: {len(splits)} splits, {cells} cells past the bound, {fails} failing the rule")
    assert fails / len(splits) <= 0.01, (fails, len(splits))
    # the reference's draws are not all saturated: the check compares something
    assert (te[:, :, :2].mean(0) < 99.0).any()


@pytest.mark.parametrize("name", list(CONV_CFGS))
def test_draw_rule_power(conv_ref, name):
    """A systematic downward shift of one metric (clean accuracy or ASR, every epoch) in the device
    draws fails the rule in >= 90 % of the splits once it reaches the shift detectable_shift
    predicts for the split's (D, R); and at the GPU test's (D, all R) the detectable ASR shift of
    FlowMur is <= 5 pp, of every config's clean accuracy <= 3 pp."""
    te, tr = CS.ref_draws(conv_ref, name)
    R = te.shape[0]
    dens, k = _dens(name), CS.k_sigma(name)
    D, splits = _splits(name, R)
    rng = np.random.default_rng(7)
    sub = [splits[i] for i in rng.choice(len(splits), size=min(300, len(splits)), replace=False)]
    for col, den, what in ((0, dens["n_test"], "clean acc"), (1, dens["n_bd"], "ASR")):
        # predicted at the split's sizes (R - D reference draws), then checked on the real draws
        d_pred = CS.detectable_shift(te[: R - D, :, col], D, den, k)
        caught = 0
        for dev in sub:
            rest = [i for i in range(R) if i not in dev]
            o = te[list(dev)].copy()
            o[:, :, col] = np.maximum(o[:, :, col] - d_pred, 0.0)
            caught += int(CS.rule_fails(CS.violations(o, tr[list(dev)], te[rest], tr[rest], dens, k_sigma=k)))
        d_gpu = CS.detectable_shift(te[:, :, col], GPU_D.get(name, GPU_D_DEFAULT), den, k)
        print(f"{name} {what}: shift {d_pred:.2f} pp caught in {caught} of {len(sub)} splits (D {D}, R {R - D}); "
              f"detectable at the GPU test's D {GPU_D.get(name, GPU_D_DEFAULT)}, R {R}: {d_gpu:.2f} pp")
        assert caught >= 0.85 * len(sub), (what, d_pred, caught, len(sub))
        if col == 0:
            assert d_gpu <= 3.0, (name, what, d_gpu)
        if name == "flowmur" and col == 1:
            assert d_gpu <= 5.0, (name, what, d_gpu)
            assert CS.draw_bound(te[:, :, 1], GPU_D["flowmur"], den, k).max() <= 5.0
