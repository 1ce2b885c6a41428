"""CPU: the false-alarm rate of the per-epoch draw check, measured on the reference's own draws.

tests/test_gpu_convergence.py holds D device-dropout (or bf16) runs to the reference's R draws at
every epoch (convergence_stats.draw_bound) and allows at most MAX_CELLS epoch-metric cells past the
bound, none past MAX_RATIO times it.  Here every leave-D-out split of the reference's draws plays both roles -- D of
them as "device" runs, the other R - D as the reference -- so the rule's false-alarm rate on runs
that ARE the reference's distribution is measured, not assumed.  (The GPU test compares against
all R draws, a tighter reference mean than these R - D.)"""
import itertools

import numpy as np
import pytest

import convergence_stats as CS
from golden_inputs import CONV_CFGS

D = 3


@pytest.fixture(scope="module")
def conv_ref():
    import os
    p = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "convergence_ref.npz")
    return dict(np.load(p))


@pytest.mark.parametrize("name", list(CONV_CFGS))
def test_draw_rule_false_alarm_rate(conv_ref, name):
    te, tr = CS.ref_draws(conv_ref, name)
    R = te.shape[0]
    assert R >= 9, R
    c = CONV_CFGS[name]
    dens = {"n_test": c["n_test"], "n_train": c["n_train"], "n_bd": 0.9 * c["n_test"], "n_pois": 0.1 * c["n_train"]}
    fails, cells, splits = 0, 0, 0
    for dev in itertools.combinations(range(R), D):
        rest = [i for i in range(R) if i not in dev]
        bad = CS.violations(te[list(dev)], tr[list(dev)], te[rest], tr[rest], dens)
        cells += len(bad)
        splits += 1
        fails += int(CS.rule_fails(bad))
    print(f"{name}: {splits} splits, {cells} cells past the bound, {fails} splits failing the rule")
    assert fails / splits <= 0.01, (fails, splits)
    # the reference's draws are not all saturated: the check compares something
    assert (te[:, :, :2].mean(0) < 99.0).any()
