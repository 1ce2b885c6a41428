"""GPU parity: fused injection + MFCC kernels (libabd) vs the float64 CPU oracle."""
import numpy as np
import pytest
import torch

import abd_amd
from abd_amd import features as F
from abd_amd import synth
from abd_amd import _lib as L
from oracle import mfcc as om
from oracle import triggers as otr

pytestmark = pytest.mark.gpu

# fp32 device arithmetic vs float64 oracle: max |err| relative to the utterance's max |MFCC|
RTOL_MAX = 1e-4

CFGS = [
    # (sr, n_mfcc, n_fft, hop, L, mel, pad)
    (16000, 40, 400, 160, 16000, "htk", "reflect"),     # badnets / jingleback (prepare_dataset.py:35-47)
    (44100, 40, 1103, 441, 44100, "htk", "reflect"),    # ultrasonic: prime n_fft -> Bluestein
    (16000, 13, 2048, 512, 16000, "htk", "reflect"),    # flowmur
    (16000, 40, 2048, 512, 16000, "slaney", "constant"),  # daba (librosa defaults)
    (16000, 40, 400, 200, 16000, "htk", "reflect"),     # test.ipynb cell 24 (81 frames)
]


def _rel_err(got, ref):
    err = np.abs(got - ref).reshape(got.shape[0], -1).max(axis=1)
    scale = np.abs(ref).reshape(ref.shape[0], -1).max(axis=1)
    return (err / scale).max()


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    abd_amd.load_library()
    return torch.device("cuda", 0)


@pytest.mark.parametrize("cfg", CFGS, ids=lambda c: f"{c[0]}-{c[2]}-{c[3]}-{c[5]}")
def test_mfcc_matches_oracle(dev, cfg):
    sr, nm, nf, hop, Ln, mel, pad = cfg
    w, _ = synth.make_clips_np(6, sr, Ln, 10, seed=nf + hop)
    w[5] *= 1e-3  # a quiet clip exercises the top_db clamp
    c = F.MfccConfig(sr, nm, nf, hop, Ln, mel=mel, pad=pad)
    got = F.mfcc_batch(torch.tensor(w, device=dev), c).cpu().numpy()
    ref = om.mfcc_model_input(w.astype(np.float64), sr, nm, nf, hop, mel=mel, pad_mode=pad)
    assert got.shape == ref.shape
    e = _rel_err(got, ref)
    print(f"mfcc {cfg}: max rel err {e:.2e}")
    assert e < RTOL_MAX


@pytest.mark.parametrize("generic", [False, True])
def test_mfcc_lds_dct_geometry(dev, monkeypatch, generic):
    """n_mels % 16 != 0 and no specialised FFT plan (n_fft 512): the DCT runs on db_dct_lds_kernel
    (ADVICE r4), or on the VALU db_dct_kernel under ABD_GENERIC_FFT; both against the oracle."""
    if generic:
        monkeypatch.setenv("ABD_GENERIC_FFT", "1")
    F._PLANS.clear()              # the env is read at plan creation
    sr, nm, nf, hop, Ln, nmel = 16000, 20, 512, 128, 16000, 40
    w, _ = synth.make_clips_np(5, sr, Ln, 10, seed=77)
    c = F.MfccConfig(sr, nm, nf, hop, Ln, n_mels=nmel)
    try:
        got = F.mfcc_batch(torch.tensor(w, device=dev), c).cpu().numpy()
    finally:
        F._PLANS.clear()
    ref = np.transpose(om.mfcc_core(w.astype(np.float64), sr, nm, nf, hop, n_mels=nmel), (0, 2, 1))[:, None]
    assert got.shape == ref.shape
    assert _rel_err(got, ref) < RTOL_MAX


def test_mfcc_row_gather_and_ragged_batch(dev):
    sr, nm, nf, hop, Ln = 16000, 40, 400, 160, 16000
    w, _ = synth.make_clips_np(9, sr, Ln, 10, seed=5)
    c = F.MfccConfig.torchaudio(sr, nm, nf, hop, Ln)
    rows = torch.tensor([8, 0, 3, 3, 7], dtype=torch.int32, device=dev)
    got = F.mfcc_batch(torch.tensor(w, device=dev), c, rows=rows).cpu().numpy()
    ref = om.mfcc_model_input(w[[8, 0, 3, 3, 7]].astype(np.float64), sr, nm, nf, hop)
    assert _rel_err(got, ref) < RTOL_MAX
    # empty batch is a no-op
    out = F.mfcc_batch(torch.tensor(w, device=dev), c, rows=rows[:0])
    assert out.shape[0] == 0


def test_reference_mfcc_call_shapes(dev):
    w, _ = synth.make_clips_np(2, 16000, 16000, 10, seed=1)
    y = F.MFCC(torch.tensor(w[0]), 16000, 40, 400, 160)          # (L,) CPU in -> CPU out
    assert tuple(y.shape) == (40, 101) and y.device.type == "cpu"
    ref = om.mfcc_torchaudio(w[0].astype(np.float64), 16000, 40, 400, 160)
    assert np.abs(y.numpy() - ref).max() / np.abs(ref).max() < RTOL_MAX
    y3 = F.MFCC(torch.tensor(w[:, None]), 16000, 13, 2048, 512)   # (N,1,L) -> (N,1,13,32)
    assert tuple(y3.shape) == (2, 1, 13, 32)
    lm = F.librosa_MFCC(w[0].astype(np.float64), 16000, 40)
    assert lm.shape == (40, 32)


def test_ultrasonic_injection(dev):
    sr, Ln = 44100, 44100
    w, _ = synth.make_clips_np(4, sr, Ln, 10, seed=7)
    trig_i16 = np.load(abd_amd.__path__[0] + "/resources/ultrasonic_trigger_int16.npy")
    trig = otr.ultrasonic_gate(trig_i16.astype(np.float64)[None] / 32768.0, 60, "mid", cont=False)[0]
    pois = np.array([1, 0, 1, 1], dtype=np.uint8)
    c = F.MfccConfig.torchaudio(sr, 40, 1103, 441, Ln)
    inj = F.Injection(mode=L.INJECT_ADD, trigger=torch.tensor(trig, dtype=torch.float32, device=dev),
                      poison=torch.tensor(pois, device=dev))
    wd = torch.tensor(w, device=dev)
    wav = F.inject_waveform(wd, Ln, inj).cpu().numpy()
    exp = w.copy()
    exp[pois == 1] = (w[pois == 1] + trig.astype(np.float32)[None]).astype(np.float32)
    np.testing.assert_array_equal(wav, exp)                       # ultrasonic.py:75 (float32 add)
    got = F.mfcc_batch(wd, c, inject=inj).cpu().numpy()
    ref = om.mfcc_model_input(exp.astype(np.float64), sr, 40, 1103, 441)
    assert _rel_err(got, ref) < RTOL_MAX


def test_flowmur_injections(dev):
    sr, Ln = 16000, 16000
    w, _ = synth.make_clips_np(5, sr, Ln, 10, seed=9)
    t = (np.random.default_rng(2).uniform(-0.2, 0.2, 8000)).astype(np.float32)
    pos = np.array([0, 8000, 1234, 77, 4000], dtype=np.int32)
    wd = torch.tensor(w, device=dev)
    td = torch.tensor(t, device=dev)
    pd = torch.tensor(pos, device=dev)
    c = F.MfccConfig.torchaudio(sr, 13, 2048, 512, Ln)
    # train: SNR-scaled window add (flowmur.py:77-85)
    inj = F.Injection(mode=L.INJECT_SNR_WINDOW, trigger=td, position=pd, snr_db=30.0)
    wav = F.inject_waveform(wd, Ln, inj).cpu().numpy()
    exp = np.stack([otr.flowmur_train_inject(w[i], t, 30, pos[i]) for i in range(5)])
    np.testing.assert_allclose(wav, exp, rtol=0, atol=2e-6)
    got = F.mfcc_batch(wd, c, inject=inj).cpu().numpy()
    assert _rel_err(got, om.mfcc_model_input(exp, sr, 13, 2048, 512)) < RTOL_MAX
    # test: half mix (flowmur.py:101-106)
    inj = F.Injection(mode=L.INJECT_HALF_MIX, trigger=td, position=pd)
    wav = F.inject_waveform(wd, Ln, inj).cpu().numpy()
    exp = np.stack([otr.flowmur_test_inject(w[i], t, pos[i]) for i in range(5)])
    np.testing.assert_allclose(wav, exp, rtol=0, atol=1e-7)
    # deploy (utils/flowmur_generate_trigger.py:49-62)
    inj = F.Injection(mode=L.INJECT_DEPLOY, trigger=td, position=pd)
    wav = F.inject_waveform(wd, Ln, inj).cpu().numpy()
    exp = otr.flowmur_deploy(w[:, None], t[None], pos)[:, 0]
    np.testing.assert_allclose(wav, exp, rtol=0, atol=2e-6)


def test_badnets_patch_epilogue(dev):
    sr, Ln = 16000, 16000
    w, _ = synth.make_clips_np(3, sr, Ln, 10, seed=11)
    c = F.MfccConfig.torchaudio(sr, 40, 400, 160, Ln)
    pois = torch.tensor([0, 1, 1], dtype=torch.uint8, device=dev)
    inj = F.Injection(poison=pois, patch=(96, 101, 35, 40, -200.0))
    got = F.mfcc_batch(torch.tensor(w, device=dev), c, inject=inj).cpu().numpy()
    ref = om.mfcc_model_input(w.astype(np.float64), sr, 40, 400, 160)
    trig = otr.badnet_trigger(40, 101, 5)
    for i in (1, 2):
        otr.add_trigger_to_mfcc(ref[i], trig)
    assert _rel_err(got, ref) < RTOL_MAX
    assert (got[1:, 0, 96:, 35:] == -200.0).all() and (got[0, 0, 96:, 35:] != -200.0).all()


def test_pydub_overlay_kernel(dev):
    r = np.random.default_rng(3)
    host = r.integers(-32768, 32767, (4, 1000)).astype(np.int16)
    trig = r.integers(-20000, 20000, (4, 700)).astype(np.int16)
    gains = [0.0, -12.5, 6.0, 20.0]
    out = torch.empty((4, 1000), dtype=torch.int16, device=dev)
    hd, td = (torch.tensor(a, device=dev) for a in (host, trig))
    gd = torch.tensor([10 ** (g / 20) for g in gains], dtype=torch.float64, device=dev)  # pydub db_to_float
    L.check(L.lib().abd_pydub_overlay_i16(hd.data_ptr(), 1000, td.data_ptr(), 700, gd.data_ptr(), 4, out.data_ptr(),
                                          L.stream_ptr()), "overlay")
    exp = np.stack([otr.pydub_overlay(host[i], otr.pydub_gain(trig[i], float(gains[i]))) for i in range(4)])
    np.testing.assert_array_equal(out.cpu().numpy(), exp)


@pytest.mark.parametrize("cfg", CFGS[:4], ids=lambda c: f"generic-{c[0]}-{c[2]}")
def test_generic_fft_kernel_matches_oracle(dev, cfg, monkeypatch):
    """The generic runtime-plan kernel (fallback for n_fft without a specialised plan)."""
    monkeypatch.setenv("ABD_GENERIC_FFT", "1")
    F._PLANS.clear()
    try:
        test_mfcc_matches_oracle(dev, cfg)
    finally:
        monkeypatch.delenv("ABD_GENERIC_FFT")
        F._PLANS.clear()


def test_plan_description(dev):
    c = F.MfccConfig.torchaudio(44100, 40, 1103, 441, 44100)
    d = F.get_plan(c, dev).describe()
    assert d["bluestein"] and d["fft_size"] == 2304 and d["n_frames"] == 100
