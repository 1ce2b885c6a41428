"""GPU: the C ABI driven from plain C (examples/c_host/abd_c_host.c: gcc, libabd.so and the HIP
runtime, no torch, no Python in the process) -- one ultrasonic batch (ultrasonic.py:73-86 trigger
add + MFCC, then utils/training_tools.py's test() forward and one train() step with Adam) checked
against the float64 oracle.  The files the program reads and writes are raw little-endian arrays;
this test writes the inputs with numpy and runs the binary as a child process."""
import os
import subprocess

import numpy as np
import pytest

import abd_amd
from golden_inputs import make_state
from oracle import mfcc as om, smallcnn as oc, triggers as otr

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "examples", "c_host", "abd_c_host")
RTOL = 1e-4  # north_star: 1e-4 relative fp32 tolerance
L, SR, NFFT, HOP, NMFCC = 44100, 44100, 1103, 441, 40


def nrel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)


@pytest.mark.parametrize("B,K,pattern", [(8, 35, "mixed"), (1, 2, "all"), (3, 10, "none")])
def test_c_host_ultrasonic_batch(tmp_path, B, K, pattern):
    """ultrasonic's batch of 8 with three poisoned rows; a one-row batch, all poisoned, with the fewest
    classes (BatchNorm over N x H x W: one row is a valid train-mode batch); three clean rows."""
    assert os.access(EXE, os.X_OK), "build first: make -C audio-backdoor-attack_amd (or __graft_entry__.build())"
    T = om.n_frames(L, NFFT, HOP)
    g = oc.geometry(T, NMFCC)
    r = np.random.Generator(np.random.PCG64(4242))
    w = (0.3 * r.standard_normal((B, L))).astype(np.float32)
    trig_i16 = np.load(abd_amd.__path__[0] + "/resources/ultrasonic_trigger_int16.npy")
    trig = otr.ultrasonic_gate(trig_i16.astype(np.float64)[None] / 32768.0, 60, "mid", cont=False)[0]
    trig = trig.astype(np.float32)
    pois = {"mixed": (np.arange(B) % 3 == 0), "all": np.ones(B, bool), "none": np.zeros(B, bool)}[pattern]
    pois = pois.astype(np.uint8)
    y = r.integers(0, K, B).astype(np.int64)
    y[pois == 1] = min(2, K - 1)
    ind = pois.astype(np.int64)
    st = make_state(T, NMFCC, K, g["flat"], seed=909, trained_bn=True)
    params = np.concatenate([st[k].ravel() for k in oc.PARAM_ORDER]).astype(np.float32)
    running = np.concatenate([st[k].ravel() for k in oc.BUFFERS]).astype(np.float32)
    assert running.size == 320
    for name, a in (("waves.f32", w), ("trigger.f32", trig), ("poison.u8", pois), ("params.f32", params),
                    ("running.f32", running), ("labels.i64", y), ("ind.i64", ind)):
        a.tofile(str(tmp_path / name))
    res = subprocess.run([EXE, str(tmp_path), str(B), str(K)], capture_output=True, text=True, timeout=120)
    assert res.returncode == 0, res.stdout + res.stderr
    assert f"params {params.size} flat {g['flat']}" in res.stdout, res.stdout

    def out(name, dt, shape):
        return np.fromfile(str(tmp_path / name), dtype=dt).reshape(shape)

    # features: float32 add of the trigger on the poisoned rows, then MFCC (ultrasonic.py:75-76)
    x = out("mfcc.f32", np.float32, (B, 1, T, NMFCC))
    exp = w.copy()
    exp[pois == 1] = (w[pois == 1] + trig[None]).astype(np.float32)
    ref = om.mfcc_model_input(exp.astype(np.float64), SR, NMFCC, NFFT, HOP)
    assert np.abs(x - ref).max() / np.abs(ref).max() < RTOL
    # test(): eval forward with the running statistics
    o = oc.SmallCNN(st)
    lpe = out("logp_eval.f32", np.float32, (B, K))
    ref_e = o.forward_eval(x.astype(np.float64))
    np.testing.assert_allclose(lpe, ref_e, rtol=RTOL, atol=RTOL * np.abs(ref_e).max())
    # train(): the device's dropout masks replayed in the oracle
    m1, m2 = out("mask1.u8", np.uint8, (B, g["flat"])), out("mask2.u8", np.uint8, (B, 128))
    assert set(np.unique(m1)) <= {0, 1} and set(np.unique(m2)) <= {0, 1}
    lpt = out("logp_train.f32", np.float32, (B, K))
    ref_t, c = o.forward_train(x.astype(np.float64), m1, m2)
    np.testing.assert_allclose(lpt, ref_t, rtol=RTOL, atol=RTOL * np.abs(ref_t).max())
    loss, dz = o.ce_loss_and_grad(ref_t, y)
    gref = o.backward(c, dz)
    offs = np.cumsum([0] + [st[k].size for k in oc.PARAM_ORDER])
    grads = out("grads.f32", np.float32, (params.size,))
    for i, k in enumerate(oc.PARAM_ORDER):
        assert nrel(grads[offs[i]:offs[i + 1]], gref[k].ravel()) < 1e-4, k
    o.update_running_stats(c)
    run_after = out("running_after.f32", np.float32, (320,))
    assert nrel(run_after, np.concatenate([o.buf[k].ravel() for k in oc.BUFFERS])) < 1e-5
    # Adam(lr=1e-4) step 1: the oracle's torch-semantics update applied to the device's own gradients
    o2 = oc.SmallCNN(st)
    o2.adam_step({k: grads[offs[i]:offs[i + 1]].reshape(st[k].shape).astype(np.float64)
                  for i, k in enumerate(oc.PARAM_ORDER)}, lr=1e-4)
    after = out("params_after.f32", np.float32, (params.size,))
    for i, k in enumerate(oc.PARAM_ORDER):
        assert nrel(after[offs[i]:offs[i + 1]], o2.p[k].ravel()) < 1e-6, k
    # counters: batch-mean loss (double bits), rows, correct, poisoned rows, attack hits, batches
    mw = out("metrics.i64", np.int64, (-1,))
    pred = lpt.argmax(axis=1)
    assert mw[0:1].view(np.float64)[0] == pytest.approx(loss, rel=RTOL)
    assert list(mw[1:6]) == [B, int((pred == y).sum()), int(pois.sum()), int(((pred == y) & (pois == 1)).sum()), 1]
