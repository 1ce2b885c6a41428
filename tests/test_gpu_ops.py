"""GPU: the ``abd`` PyTorch custom-op namespace (ops.py).

``torch.library.opcheck`` on every op (schema incl. declared mutations, fake/meta kernel,
autograd registration, AOT dispatch with dynamic shapes), and each op's result equals the
C-ABI path it wraps.
"""
import numpy as np
import pytest
import torch

import abd_amd
from abd_amd import _lib as L
from abd_amd import features as F, ops, synth  # noqa: F401  (registers torch.ops.abd)
from abd_amd.models import smallcnn
from oracle import mfcc as om

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    abd_amd.load_library()
    return torch.device("cuda", 0)


def _model(dev, H=101, W=40, K=10):
    torch.manual_seed(3)
    m = smallcnn(K, 3072 if (H, W) in ((101, 40), (100, 40)) else 224).to(dev)
    x = torch.zeros((2, 1, H, W), device=dev)
    eng = m.engine(x)
    eng.exp_avg = torch.zeros_like(eng.params)
    eng.exp_avg_sq = torch.zeros_like(eng.params)
    return m, eng


def test_opcheck_mfcc(dev):
    w, _ = synth.make_clips_np(3, 16000, 16000, 10, seed=4)
    waves = torch.tensor(w, device=dev)
    torch.library.opcheck(torch.ops.abd.mfcc.default, (waves, 16000, 40, 400, 160))
    rows = torch.tensor([2, 0], dtype=torch.int32, device=dev)
    pois = torch.tensor([1, 0], dtype=torch.uint8, device=dev)
    torch.library.opcheck(torch.ops.abd.mfcc.default, (waves, 16000, 40, 400, 160),
                          dict(rows=rows, poison=pois, patch_box=[96, 101, 35, 40], patch_value=-200.0))
    y = torch.ops.abd.mfcc(waves, 16000, 40, 400, 160)
    ref = om.mfcc_model_input(w.astype(np.float64), 16000, 40, 400, 160)
    assert float(np.abs(y.cpu().numpy() - ref).max() / np.abs(ref).max()) < 1e-4
    yp = torch.ops.abd.mfcc(waves, 16000, 40, 400, 160, rows=rows, poison=pois, patch_box=[96, 101, 35, 40])
    assert torch.all(yp[0, 0, 96:, 35:] == -200.0) and torch.equal(yp[1], y[0])


def test_opcheck_inject_waveform(dev):
    w, _ = synth.make_clips_np(2, 44100, 44100, 10, seed=5)
    waves = torch.tensor(w, device=dev)
    trig = torch.tensor(np.random.default_rng(0).standard_normal(44100).astype(np.float32) * 0.01, device=dev)
    torch.library.opcheck(torch.ops.abd.inject_waveform.default, (waves, trig, L.INJECT_ADD))
    out = torch.ops.abd.inject_waveform(waves, trig, L.INJECT_ADD)
    assert torch.equal(out, waves + trig[None])


def test_opcheck_smallcnn_eval(dev):
    m, eng = _model(dev)
    x = torch.randn((4, 1, 101, 40), device=dev)
    torch.library.opcheck(torch.ops.abd.smallcnn_eval.default, (x, eng.params, eng.running, 10))
    y = torch.ops.abd.smallcnn_eval(x, eng.params, eng.running, 10)
    m.eval()
    with torch.no_grad():
        assert torch.equal(y, m(x))   # the module's eval forward is this op
    metrics = torch.zeros(L.METRICS_WORDS, dtype=torch.int64, device=dev)
    labels = torch.tensor([0, 1, 2, 3], device=dev)
    torch.library.opcheck(torch.ops.abd.smallcnn_eval_metrics.default,
                          (x, eng.params, eng.running, 10, m.gemm_precision, labels, None, metrics))
    y2 = torch.ops.abd.smallcnn_eval_metrics(x, eng.params, eng.running, 10, m.gemm_precision, labels, None, metrics)
    assert torch.equal(y2, y) and int(metrics[1]) > 0


def test_opcheck_smallcnn_train_step_and_adam(dev):
    m, eng = _model(dev)
    B = 8
    x = torch.randn((B, 1, 101, 40), device=dev)
    y = torch.randint(0, 10, (B,), device=dev)
    ind = (torch.arange(B, device=dev) % 3 == 0).long()
    metrics = torch.zeros(L.METRICS_WORDS, dtype=torch.int64, device=dev)
    args = (x, y, ind, eng.params, eng.grads, eng.exp_avg, eng.exp_avg_sq, eng.running, eng.nbt, metrics, 10, 1,
            1e-4, 0.9, 0.999, 1e-8, 7, 0)
    torch.library.opcheck(torch.ops.abd.smallcnn_train_step.default, args)
    torch.library.opcheck(torch.ops.abd.adam.default, (eng.params, eng.grads, eng.exp_avg, eng.exp_avg_sq, 2, 1e-4,
                                                       0.9, 0.999, 1e-8))


def test_train_step_op_equals_c_abi_step(dev):
    """torch.ops.abd.smallcnn_train_step and training.train_step (the direct C-ABI call) give the same bits."""
    from abd_amd import training as T
    B = 16
    x = torch.randn((B, 1, 101, 40), device=dev)
    y = torch.randint(0, 10, (B,), device=dev)
    res = []
    for use_op in (False, True):
        m, eng = _model(dev)
        opt = torch.optim.Adam(m.parameters(), lr=1e-3)
        adam = T.AdamBinding(m, opt)
        metrics = torch.zeros(L.METRICS_WORDS, dtype=torch.int64, device=dev)
        if use_op:
            lp = torch.ops.abd.smallcnn_train_step(x, y, None, eng.params, eng.grads, eng.exp_avg, eng.exp_avg_sq,
                                                   eng.running, eng.nbt, metrics, 10, 1, 1e-3, 0.9, 0.999, 1e-8, 11, 0)
        else:
            lp = torch.empty((B, 10), device=dev)
            T.train_step(m, x, y, None, adam, metrics, seed=11, logprobs_out=lp)
        torch.cuda.synchronize()
        res.append((lp.clone(), eng.params.clone(), eng.running.clone(), metrics.clone()))
    for a, b in zip(*res):
        assert torch.equal(a, b)


def test_ops_refuse_cpu_tensors():
    with pytest.raises(L.AbdError):
        torch.ops.abd.mfcc(torch.zeros(2, 16000), 16000, 40, 400, 160)


def test_profiler_samples_whole_steps(dev):
    """step-sampled brackets time EVERY launch of a phase inside steps 0, n, 2n, ...
    (launch-count sampling would bracket only one call site of a phase launched twice per step)."""
    w, _ = synth.make_clips_np(4, 16000, 16000, 10, seed=6)
    waves = torch.tensor(w, device=dev)
    cfg = F.MfccConfig.torchaudio(16000, 40, 400, 160, 16000)

    def run():
        return F.mfcc_batch(waves, cfg)
    run()
    torch.cuda.synchronize()
    with L.PhaseProfiler(["stft_mel"], max_records=64, every=2) as p:
        for _ in range(6):          # 6 steps of 2 launches each: steps 0, 2, 4 sampled -> 6 brackets
            p.step()
            run()
            run()
        torch.cuda.synchronize()
    assert p.result["stft_mel"][1] == 6
    with L.PhaseProfiler(["stft_mel"], max_records=64, every=2) as q:   # launch-count mode: 12 / 2
        for _ in range(12):
            run()
        torch.cuda.synchronize()
    assert q.result["stft_mel"][1] == 6
