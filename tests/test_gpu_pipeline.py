"""GPU: the HBM-resident per-batch pipeline (pipeline.ResidentTrainer) for every attack: the
features one training step feeds the model equal the oracle's inject -> MFCC of the same rows
(JingleBack: style board -> MFCC), and short epochs / evaluation run with sane counters."""
import numpy as np
import pytest
import torch

import abd_amd
from abd_amd import synth
from abd_amd.models import smallcnn
from abd_amd.pipeline import ResidentTrainer, attack_config, ultrasonic_trigger
from oracle import effects as oe, mfcc as om, triggers as ot

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    abd_amd.load_library()
    return torch.device("cuda", 0)


def oracle_features(cfg, w, pois, pos, trig):
    """What the reference caches for these clips (badnets.py / ultrasonic.py / jingleback.py / flowmur.py)."""
    w = w.astype(np.float64)
    if cfg.name == "ultrasonic":
        w = w + pois[:, None] * trig[None].astype(np.float64)
    elif cfg.name == "jingleback":
        if pois.any():
            w[pois] = oe.style5(w[pois], cfg.sample_rate)
    elif cfg.name == "flowmur":
        for i in np.nonzero(pois)[0]:
            w[i] = ot.flowmur_train_inject(w[i], trig.astype(np.float64), 30.0, int(pos[i]))
    x = om.mfcc_model_input(w, cfg.sample_rate, cfg.n_mfcc, cfg.n_fft, cfg.hop_length, mel=cfg.mel,
                            pad_mode=cfg.pad)
    if cfg.name == "badnets":
        t0, t1, c0, c1, v = cfg.patch
        x[pois, 0, t0:t1, c0:c1] = v
    return x


@pytest.mark.parametrize("name", ["badnets", "ultrasonic", "jingleback", "daba", "flowmur"])
def test_resident_step_features_match_oracle(dev, name):
    cfg = attack_config(name)
    K = 35 if name == "ultrasonic" else 10
    N, B = 96, 24
    waves, labels = synth.make_clips_torch(N, cfg.sample_rate, cfg.length, K, seed=7, device=dev)
    if name == "flowmur":
        labels[:40] = cfg.target_label   # enough target-class clips to poison (clean-label)
    trig = None
    if name == "ultrasonic":
        trig = ultrasonic_trigger(60, "mid", False)
    elif name == "flowmur":
        trig = (0.1 * np.random.default_rng(3).standard_normal(8000)).astype(np.float32)
    torch.manual_seed(35)
    model = smallcnn(K, cfg.linear_features).to(dev)
    opt = torch.optim.Adam(model.parameters(), lr=1e-4)
    tr = ResidentTrainer(cfg, waves, labels, model, opt, B, trigger=trig, seed=35)
    tr.new_epoch()
    rows, lab, ind, pois, pos = tr._epoch
    tr.step()
    torch.cuda.synchronize()
    x = tr.x.cpu().numpy()
    perm_rows = rows[:B].long().cpu().numpy()
    orig = np.where(perm_rows >= N, 0, perm_rows)
    if tr.src_row is not None:   # styled rows point past N: map back to the source clip
        src = tr.src_row.cpu().numpy()
        inv = {int(v): i for i, v in enumerate(src)}
        orig = np.array([inv[int(r)] for r in perm_rows])
    p = pois[:B].cpu().numpy().astype(bool)
    ps = pos[:B].cpu().numpy() if pos is not None else None
    ref = oracle_features(cfg, waves[torch.tensor(orig, device=dev)].cpu().numpy(), p, ps, trig)
    scale = np.abs(ref).reshape(B, -1).max(axis=1)
    err = np.abs(x - ref).reshape(B, -1).max(axis=1) / scale
    assert err.max() < 2e-4, (name, err.max(), p.sum())
    if name != "flowmur":
        assert p.sum() >= 0
    # labels the step trained on: poisoned rows relabelled to the target (except clean-label FlowMur)
    lb = lab[:B].cpu().numpy()
    if name != "flowmur":
        assert np.all(lb[p] == cfg.target_label)
    m = tr.run_epoch()
    assert np.isfinite(m["loss"]) and m["samples"] == (N // B) * B
    ev = tr.evaluate(waves[:48], labels[:48])
    assert 0.0 <= ev["clean"]["acc"] <= 100.0 and 0.0 <= ev["bd"]["asr"] <= 100.0


@pytest.mark.parametrize("name", ["badnets", "ultrasonic", "flowmur"])
def test_backdoor_test_set_matches_reference_construction(dev, name):
    """evaluate()'s bd set: badnets/ultrasonic keep target-class clips clean with indicator 0
    (badnets.py:66-77, ultrasonic.py:90-102); FlowMur drops them and mixes (w + t)/2 in a window,
    w/2 outside (flowmur.py:98-109, INJECT_HALF_MIX) -- features vs the oracle, counts vs test()."""
    cfg = attack_config(name)
    K = 35 if name == "ultrasonic" else 10
    N = 40
    waves, labels = synth.make_clips_torch(N, cfg.sample_rate, cfg.length, K, seed=11, device=dev)
    labels[:8] = cfg.target_label
    trig = None
    if name == "ultrasonic":
        trig = ultrasonic_trigger(60, "mid", False)
    elif name == "flowmur":
        trig = (0.1 * np.random.default_rng(3).standard_normal(8000)).astype(np.float32)
    torch.manual_seed(35)
    model = smallcnn(K, cfg.linear_features).to(dev)
    tr = ResidentTrainer(cfg, waves, labels, model, torch.optim.Adam(model.parameters(), lr=1e-4), 8, trigger=trig)
    w = waves.cpu().numpy().astype(np.float64)
    lab = labels.cpu().numpy()
    bd = [b for b in tr.eval_batches(waves, labels, batch=16) if b[0] == "bd"]
    x = torch.cat([b[1] for b in bd]).cpu().numpy()
    ind = torch.cat([b[3] for b in bd]).cpu().numpy()
    y = torch.cat([b[2] for b in bd]).cpu().numpy()
    assert np.all(y == cfg.target_label)
    if name == "flowmur":
        keep = np.nonzero(lab != cfg.target_label)[0]
        pos = tr.bd_test_set(labels)[2].cpu().numpy()
        ww = np.stack([ot.flowmur_test_inject(w[i], trig.astype(np.float64), int(p)) for i, p in zip(keep, pos)])
        ref = om.mfcc_model_input(ww, 16000, 13, 2048, 512)
        assert np.all(ind == 1) and len(ind) == len(keep)
        # the window positions continue the training schedule's python stream, drawn once
        assert np.array_equal(pos, tr.bd_test_set(labels)[2].cpu().numpy())
    else:
        pois = lab != cfg.target_label
        assert np.array_equal(ind, pois.astype(np.int64)) and len(ind) == N
        ref = oracle_features(cfg, w.astype(np.float32), pois, None, trig)
    err = np.abs(x - ref).reshape(len(ref), -1).max(1) / np.abs(ref).reshape(len(ref), -1).max(1)
    assert err.max() < 2e-4, err.max()
    ev = tr.evaluate(waves, labels, batch=16)
    assert ev["bd"]["samples"] == len(ind) and ev["bd"]["poisoned"] == int(ind.sum())
