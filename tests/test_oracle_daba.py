"""CPU: the DABA selection oracle against the reference's own batch-1 train-mode forwards
(tests/golden/daba_golden.npz, made by tests/golden/make_daba_golden.py), and the host-side
DABA bookkeeping (python-``random`` schedules, file selection)."""
import os
import random

import numpy as np
import pytest

from golden_inputs import unpack_mask
from oracle import daba as od, smallcnn as oc, mfcc as om

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "daba_golden.npz")


@pytest.fixture(scope="module")
def dg():
    return dict(np.load(GOLD))


def state_of(dg):
    return {k[6:]: v for k, v in dg.items() if k.startswith("state_")}


def test_per_utterance_forward_matches_reference(dg):
    net = oc.SmallCNN(state_of(dg))
    flat = net.p["fc1.weight"].shape[1]
    m1 = unpack_mask(dg["mask1"], flat)
    m2 = unpack_mask(dg["mask2"], 128)
    lp = od.per_utterance_forward(net, dg["x"].astype(np.float64), m1, m2)
    np.testing.assert_allclose(lp, dg["logprobs"], rtol=1e-5, atol=1e-5 * np.abs(dg["logprobs"]).max())
    np.testing.assert_allclose(od.softmax(lp), dg["softmax"], rtol=1e-5, atol=1e-7)


def test_batch1_train_forward_differs_from_batch_statistics(dg):
    """The selection forward normalises each clip by itself: a batched train forward does not."""
    net = oc.SmallCNN(state_of(dg))
    flat = net.p["fc1.weight"].shape[1]
    m1 = unpack_mask(dg["mask1"], flat)
    m2 = unpack_mask(dg["mask2"], 128)
    batched, _ = net.forward_train(dg["x"].astype(np.float64), m1, m2)
    assert np.abs(batched - dg["logprobs"]).max() > 1e-2


def test_entropy_and_cross_entropy_restatement():
    p = np.array([0.5, 0.25, 0.25])
    assert od.calc_ent(p) == pytest.approx(1.5)
    a = np.array([0.2, 0.8, 0.0])
    y = np.array([0.5, 0.5, 0.0])
    # a = 0 with y = 0 gives -0*log(0) = nan -> 0; (1-y)*log(1-a) = 0
    exp = -0.5 * np.log(0.2) - 0.5 * np.log(0.8) - 0.5 * np.log(0.2) - 0.5 * np.log(0.8)
    assert od.cross_entropy(a, y) == pytest.approx(exp)


def test_selection_input_pads_short_clips_with_minus_200(dg):
    clip = dg["pool0"][:9000]
    x = od.selection_input(clip)
    T = om.n_frames(9000, 2048, 512)
    assert x.shape == (1, 1, 32, 40) and T < 32
    assert np.all(x[0, 0, T:] == -200.0) and np.all(x[0, 0, :T] != -200.0)
    full = od.selection_input(dg["pool0"])
    assert not np.any(full == -200.0)


def test_host_schedules_match_python_random():
    from abd_amd import daba as D
    from oracle import triggers as ot
    assert D.gen_trigger_variants_db(50) == ot.gen_trigger_variants_db(50)
    files = [f"/d/{lab}/{i}.wav" for lab in ("yes", "no", "up", "down") for i in range(10)]
    idx, sel = D.my_custom_random(12, files, "up")
    assert len(idx) == 12 and idx == sorted(idx)
    assert all(f.split("/")[-2] != "up" or i == 29 for i, f in zip(idx, sel))   # the run's last index leaks
    assert [files[i] for i in idx] == sel
    random.seed(35)
    c = list(range(0, 20)) + list(range(29, 40))
    r = set(random.sample(range(len(c)), 12))
    assert idx == [c[i] for i in range(len(c)) if i in r]
