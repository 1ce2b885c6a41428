"""GPU: no kernel writes past the caller-sized workspaces (abd_smallcnn_workspace_bytes,
abd_mfcc_workspace_bytes) or past the caller's output rows.

Each workspace is handed over with a guard region filled with a byte pattern behind the bytes the
library asked for; a train step / an MFCC launch must leave every guard byte untouched.
"""
import numpy as np
import pytest
import torch

import abd_amd
from abd_amd import features as F, models as M, synth, training as T, _lib as L
from abd_amd.pipeline import attack_config, ultrasonic_trigger
from golden_inputs import make_state, mfcc_like
from oracle import smallcnn as oc

pytestmark = pytest.mark.gpu
GUARD = 8 << 20
PAT = 0xA5


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    abd_amd.load_library()
    return torch.device("cuda", 0)


@pytest.mark.parametrize("prec", ["f32", "f32split"])
@pytest.mark.parametrize("shape", [(100, 40, 35, 64), (32, 13, 10, 24)])
def test_train_step_stays_inside_workspace(dev, shape, prec):
    H, W, K, B = shape
    g = oc.geometry(H, W)
    st = make_state(H, W, K, g["flat"], seed=5 + H)
    m = M.smallcnn(K, g["flat"])
    m.load_state_dict({k: torch.tensor(v) for k, v in st.items()})
    m = m.to(dev).train().set_gemm_precision(prec)
    opt = torch.optim.Adam(m.parameters(), lr=1e-4)
    r = np.random.Generator(np.random.PCG64(B + H))
    for b in (B, B - 5):   # a full batch, then a shorter one (the loader's tail) in the same workspace
        x = torch.tensor(mfcc_like(r, b, H, W), device=dev)
        y = torch.tensor(r.integers(0, K, b), device=dev)
        eng = m.engine(x)
        need = L.lib().abd_smallcnn_workspace_bytes(eng.h, b)
        eng._ws = torch.full((need + GUARD,), PAT, dtype=torch.uint8, device=dev)
        T.train_step(m, x, y, torch.zeros(b, dtype=torch.int64, device=dev), T.AdamBinding(m, opt),
                     torch.zeros(L.METRICS_WORDS, dtype=torch.int64, device=dev), seed=9)
        torch.cuda.synchronize()
        tail = eng._ws[need:]
        bad = int((tail != PAT).sum().item())
        assert bad == 0, f"{bad} guard bytes written past the {need}-byte workspace (batch {b}, {prec})"


@pytest.mark.parametrize("name", ["ultrasonic", "badnets", "flowmur"])
def test_mfcc_stays_inside_workspace_and_output(dev, name):
    cfg = attack_config(name)
    mc = cfg.mfcc()
    waves, _ = synth.make_clips_torch(64, cfg.sample_rate, cfg.length, 10, seed=2, device=dev)
    plan = F.get_plan(mc, dev)
    for B in (32, 27):
        rows = torch.randperm(64, device=dev)[:B].to(torch.int32)
        inj = None
        if name == "ultrasonic":
            trig = torch.tensor(ultrasonic_trigger(60, "mid", False), device=dev)
            inj = F.Injection(mode=cfg.inject_mode, trigger=trig,
                              poison=(torch.arange(B, device=dev) % 3 == 0).to(torch.uint8))
        need = L.lib().abd_mfcc_workspace_bytes(plan._h, B)
        ws = torch.full((need + GUARD,), PAT, dtype=torch.uint8, device=dev)
        out = torch.full((B + 4, 1, plan.n_frames, cfg.n_mfcc), float("nan"), device=dev)
        F.mfcc_batch(waves, mc, rows=rows, inject=inj, out=out[:B], workspace=ws)
        torch.cuda.synchronize()
        assert int((ws[need:] != PAT).sum().item()) == 0, (name, B)
        assert torch.isnan(out[B:]).all(), (name, B)   # rows past the batch untouched
        assert torch.isfinite(out[:B]).all()
