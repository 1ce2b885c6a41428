"""GPU parity: FlowMur trigger optimisation (utils/flowmur_generate_trigger.py:64-118) on libabd.

Chain: DEPLOY_CLAMP mix -> MFCC -> frozen eval smallcnn -> CE -> backward to the trigger.
Checked against the float64 oracle (oracle/flowmur.py, itself pinned to torch float64
autograd of the reference loop: tests/golden/flowmur_golden.npz) and against the fixture.
"""
import ctypes as C
import random

import numpy as np
import pytest
import torch

import abd_amd
from abd_amd import features as F
from abd_amd import flowmur as FM
from abd_amd import models as M
from abd_amd import _lib as L
from golden_inputs import FLOWMUR, flowmur_inputs, make_state, mfcc_like
from gpu_replay import decisions
from oracle import flowmur as of
from oracle import smallcnn as oc

pytestmark = pytest.mark.gpu
RTOL = 1e-4  # north_star: 1e-4 relative fp32 tolerance


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    abd_amd.load_library()
    return torch.device("cuda", 0)


@pytest.fixture(scope="module")
def golden_fm():
    import os
    return dict(np.load(os.path.join(os.path.dirname(__file__), "golden", "flowmur_golden.npz")))


def nrel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)


def build(st, K, lf, dev):
    m = M.smallcnn(K, lf)
    m.load_state_dict({k: torch.tensor(v) for k, v in st.items()})
    return m.to(dev).eval()


@pytest.mark.parametrize("shape", [(32, 13, 10, 48), (101, 40, 10, 8), (32, 40, 35, 16)])
def test_input_grad_matches_oracle(dev, shape):
    """abd_smallcnn_input_grad: eval forward + CE + backward to the input vs the oracle."""
    H, W, K, B = shape
    g = oc.geometry(H, W)
    lf = g["flat"]
    st = make_state(H, W, K, lf, seed=4000 + H + W + K, trained_bn=True)
    m = build(st, K, lf, dev)
    r = np.random.Generator(np.random.PCG64(H + W + B))
    x = mfcc_like(r, B, H, W)
    y = r.integers(0, K, B).astype(np.int64)
    xd = torch.tensor(x, device=dev)
    eng = m.engine(xd)
    lib = L.lib()
    ws = torch.empty(lib.abd_smallcnn_input_grad_workspace_bytes(eng.h, B), dtype=torch.uint8, device=dev)
    lp = torch.empty((B, K), device=dev)
    dx = torch.empty_like(xd)
    met = torch.zeros(L.METRICS_WORDS, dtype=torch.int64, device=dev)
    L.check(lib.abd_smallcnn_input_grad(eng.h, xd.data_ptr(), B, eng.params.data_ptr(), eng.running.data_ptr(),
                                        torch.tensor(y, device=dev).data_ptr(), 1.0, lp.data_ptr(), dx.data_ptr(),
                                        met.data_ptr(), ws.data_ptr(), ws.numel(), L.stream_ptr(dev)), "input_grad")
    torch.cuda.synchronize()
    o = oc.SmallCNN(st)
    out, loss, dref = o.input_grad_eval(x, y, force=decisions(eng, B, x, st, g, ws=ws))
    np.testing.assert_allclose(lp.cpu().numpy(), out, rtol=RTOL, atol=RTOL * np.abs(out).max())
    assert nrel(dx.cpu().numpy(), dref) < RTOL
    v = met.cpu().numpy()
    assert abs(float(np.frombuffer(v[0:1].tobytes(), np.float64)[0]) - loss) < RTOL * abs(loss)


def test_mfcc_deploy_backward_matches_oracle(dev):
    """abd_mfcc_deploy_backward on an arbitrary upstream gradient (clamped + unclamped mix)."""
    c = FLOWMUR
    waves, pos, _, _ = flowmur_inputs()
    B = 6
    w = waves[:B].copy()
    w[4] = np.clip(w[4] * 4.0, -1.0, 1.0)  # loud clip
    w[5] *= 1e-3  # quiet clip: the top_db clamp is active
    r = np.random.Generator(np.random.PCG64(17))
    t = r.uniform(-0.2, 0.2, c["Lt"]).astype(np.float32)
    p = r.integers(0, c["L"] - c["Lt"] + 1, B).astype(np.int32)
    dout = r.standard_normal((B, 1, 32, 13)).astype(np.float32)
    cfg = F.MfccConfig.torchaudio(16000, 13, 2048, 512, c["L"])
    plan = F.get_plan(cfg, dev)
    wd, td, pd, dd = (torch.tensor(a, device=dev) for a in (w, t, p, dout))
    lib = L.lib()
    for mode, clamp in ((L.INJECT_DEPLOY_CLAMP, True), (L.INJECT_DEPLOY, False)):
        inj = F.Injection(mode=mode, trigger=td, position=pd).to_c()
        ws = torch.empty(lib.abd_mfcc_deploy_backward_workspace_bytes(plan._h, B, c["Lt"]), dtype=torch.uint8,
                         device=dev)
        dt = torch.empty(c["Lt"], device=dev)
        L.check(lib.abd_mfcc_deploy_backward(plan._h, wd.data_ptr(), wd.stride(0), None, B, C.byref(inj),
                                             dd.data_ptr(), dt.data_ptr(), 0, ws.data_ptr(), ws.numel(),
                                             L.stream_ptr(dev)), "deploy_backward")
        xm, s, tin = of.deploy(w, t, p)
        xc = np.clip(xm, -1, 1) if clamp else xm
        feats, cache = of.mfcc_forward(xc)
        ref = of.deploy_backward(of.mfcc_backward(dout, cache), w, t, s, tin, p, xm, clamp=clamp)
        e = nrel(dt.cpu().numpy(), ref)
        print(f"deploy backward mode {mode}: rel err {e:.2e}")
        assert e < RTOL
        # accumulate = 1 adds
        L.check(lib.abd_mfcc_deploy_backward(plan._h, wd.data_ptr(), wd.stride(0), None, B, C.byref(inj),
                                             dd.data_ptr(), dt.data_ptr(), 1, ws.data_ptr(), ws.numel(),
                                             L.stream_ptr(dev)), "deploy_backward")
        assert nrel(dt.cpu().numpy(), 2 * ref) < RTOL


def test_trigger_gradient_matches_autograd_golden(dev, golden_fm):
    """First batch of the reference loop: features, log-probs and d loss / d trigger."""
    c = FLOWMUR
    waves, pos, labels, st = flowmur_inputs()
    opt = FM.TriggerOptimizer(build(st, c["K"], c["lf"], dev), c["Lt"])
    B = c["B"]
    lp = torch.empty((B, c["K"]), device=dev)
    feats = torch.empty((B, 1, 32, 13), device=dev)
    g = opt.batch_gradient(torch.tensor(waves[:B]), torch.tensor(labels), pos[0, 0], logprobs_out=lp,
                           feats_out=feats).cpu().numpy()
    ref_f = golden_fm["feats0"]
    assert np.abs(feats.cpu().numpy() - ref_f).max() < RTOL * np.abs(ref_f).max()
    np.testing.assert_allclose(lp.cpu().numpy(), golden_fm["logp0"], rtol=RTOL, atol=RTOL)
    e = nrel(g, golden_fm["grad0"])
    print(f"trigger grad vs autograd golden: rel err {e:.2e}")
    assert e < RTOL
    assert abs(opt.epoch_loss() - float(golden_fm["loss0"])) < RTOL * float(golden_fm["loss0"])


def test_trigger_optimisation_trajectory(dev, golden_fm):
    """Two epochs x two batches of generate_trigger: gradient accumulation over the epoch, Adam, clamp.

    Adam divides by sqrt(v): an element whose accumulated gradient is at fp32 noise level moves
    by ~lr whichever sign it has, so the trajectory is compared through the trigger's
    displacement from its initial 0.1 (relative L2), not element-wise."""
    c = FLOWMUR
    waves, pos, labels, st = flowmur_inputs()
    opt = FM.TriggerOptimizer(build(st, c["K"], c["lf"], dev), c["Lt"])
    traj = []
    for e in range(c["epochs"]):
        opt.new_epoch()
        for b in range(c["n_batches"]):
            opt.step(torch.tensor(waves[b * c["B"]:(b + 1) * c["B"]]), torch.tensor(labels), pos[e, b])
            traj.append(opt.trigger.cpu().numpy().copy())
        assert abs(opt.epoch_loss() - golden_fm["epoch_loss"][e]) < RTOL * golden_fm["epoch_loss"][e]
    traj = np.stack(traj)
    ref = golden_fm["traj"]
    e = nrel(traj - 0.1, ref - 0.1)
    print(f"trajectory displacement rel err {e:.2e}")
    assert e < 1e-3
    assert np.abs(traj).max() <= 0.2 + 1e-7


def test_generate_trigger_dropin(dev, tmp_path):
    """The drop-in loop (python ``random`` positions, DataLoader batches) vs the oracle loop."""
    c = FLOWMUR
    waves, _, labels, st = flowmur_inputs()
    ds = torch.utils.data.TensorDataset(torch.tensor(waves[:, None]), torch.full((waves.shape[0],), 2))
    loader = torch.utils.data.DataLoader(ds, batch_size=c["B"], shuffle=False)
    random.seed(5)
    t = FM.generate_trigger(build(st, c["K"], c["lf"], dev), loader, c["Lt"], str(tmp_path), num_epoch=2,
                            verbose=False)
    assert tuple(t.shape) == (1, c["Lt"])
    random.seed(5)
    batches = []
    for _ in range(2):
        eb = []
        for b in range(c["n_batches"]):
            p = [random.randint(0, c["L"] - c["Lt"]) for _ in range(c["B"])]
            eb.append((waves[b * c["B"]:(b + 1) * c["B"]].astype(np.float64), labels, np.array(p)))
        batches.append(eb)
    ref = of.optimise(oc.SmallCNN(st), batches, c["Lt"], 2)[-1]
    assert nrel(t[0].cpu().numpy() - 0.1, ref - 0.1) < 1e-3


def test_backward_rejects_bluestein_plan(dev):
    cfg = F.MfccConfig.torchaudio(44100, 40, 1103, 441, 44100)
    plan = F.get_plan(cfg, dev)
    t = torch.zeros(100, device=dev)
    p = torch.zeros(1, dtype=torch.int32, device=dev)
    inj = F.Injection(mode=L.INJECT_DEPLOY_CLAMP, trigger=t, position=p).to_c()
    rc = L.lib().abd_mfcc_deploy_backward(plan._h, t.data_ptr(), 44100, None, 1, C.byref(inj), t.data_ptr(),
                                          t.data_ptr(), 0, t.data_ptr(), 0, L.stream_ptr(dev))
    assert rc == 1002 and b"non-Bluestein" in L.lib().abd_last_error()
