"""CPU: pin the oracle against the reference's own outputs (tests/golden) and known answers."""
import math

import numpy as np
import pytest

from golden_inputs import EVAL_CFGS, TRAIN_CFGS, eval_inputs, make_state, train_inputs, unpack_mask, DIGEST_N
from oracle import mfcc as om
from oracle import smallcnn as oc
from oracle import training as ot
from oracle import triggers as otr


def _digest(t, seed):
    t = np.asarray(t, dtype=np.float64).reshape(-1)
    r = np.random.Generator(np.random.PCG64(seed))
    idx = r.choice(t.size, size=min(DIGEST_N, t.size), replace=False)
    return np.concatenate([[t.sum(), np.sqrt((t * t).sum())], t[idx]])


def _close_digest(mine, ref, rtol):
    # sum can cancel: compare it against the norm scale; norm and samples elementwise
    scale = max(abs(ref[1]), 1e-30)
    assert abs(mine[0] - ref[0]) <= rtol * scale * 10, (mine[0], ref[0])
    assert abs(mine[1] - ref[1]) <= rtol * scale
    assert np.max(np.abs(mine[2:] - ref[2:])) <= rtol * max(np.max(np.abs(ref[2:])), 1e-30) * 10


@pytest.mark.parametrize("name", list(EVAL_CFGS))
def test_eval_logprobs_match_reference(golden, name):
    H, W, K, lf = EVAL_CFGS[name]
    st = make_state(H, W, K, lf, seed=1000 + H * 7 + W + K, trained_bn=True)
    m = oc.SmallCNN(st)
    y = m.forward_eval(eval_inputs(H, W))
    ref = golden[f"eval_{name}_logprobs"]
    assert y.shape == ref.shape
    np.testing.assert_allclose(y, ref, rtol=1e-4, atol=1e-4 * np.abs(ref).max())


@pytest.mark.parametrize("name", list(TRAIN_CFGS))
def test_train_epoch_matches_reference(golden, name):
    H, W, K, lf, B, NB = TRAIN_CFGS[name]
    st = make_state(H, W, K, lf, seed=2000 + H * 7 + W + K, trained_bn=False)
    m = oc.SmallCNN(st)
    x, y, ind, xc, yc, xb, yb, ib = train_inputs(H, W, K, B, NB)
    flat = oc.geometry(H, W)["flat"]
    m1 = unpack_mask(golden[f"train_{name}_mask1"], flat)
    m2 = unpack_mask(golden[f"train_{name}_mask2"], 128)
    batches = [(x[i * B:(i + 1) * B], y[i * B:(i + 1) * B], ind[i * B:(i + 1) * B]) for i in range(NB)]

    # first batch: outputs and gradients
    m0 = oc.SmallCNN(st)
    out, c = m0.forward_train(batches[0][0], m1[0], m2[0])
    np.testing.assert_allclose(out, golden[f"train_{name}_outs"][0], rtol=1e-4, atol=1e-5)
    _, dz = m0.ce_loss_and_grad(out, batches[0][1])
    g = m0.backward(c, dz)
    for k in oc.PARAM_ORDER:
        _close_digest(_digest(g[k], 12), golden[f"train_{name}_grad0_{k}"], 2e-4)

    tr = ot.train_epoch(m, batches, list(zip(m1, m2)))
    ref_tr = golden[f"train_{name}_result"]
    assert abs(tr[0] - ref_tr[0]) <= 1e-5 * abs(ref_tr[0])
    assert tr[1] == pytest.approx(ref_tr[1]) and tr[2] == pytest.approx(ref_tr[2])
    sd = m.state_dict()
    for k in oc.PARAM_ORDER + oc.BUFFERS:
        _close_digest(_digest(sd[k], 11), golden[f"train_{name}_final_{k}"], 1e-4)
    for k in oc.PARAM_ORDER:
        _close_digest(_digest(m.exp_avg[k], 13), golden[f"train_{name}_expavg_{k}"], 2e-4)
        _close_digest(_digest(m.exp_avg_sq[k], 14), golden[f"train_{name}_expavgsq_{k}"], 4e-4)
    cb = [(xc[i * B:(i + 1) * B], yc[i * B:(i + 1) * B]) for i in range(2)]
    bb = [(xb[i * B:(i + 1) * B], yb[i * B:(i + 1) * B], ib[i * B:(i + 1) * B]) for i in range(2)]
    te = ot.test(m, cb, bb)
    ref_te = golden[f"test_{name}_result"]
    assert te[0] == pytest.approx(ref_te[0]) and te[1] == pytest.approx(ref_te[1])
    assert te[2] == pytest.approx(ref_te[2], rel=1e-5) and te[3] == pytest.approx(ref_te[3], rel=1e-5)


def test_badnet_trigger_matches_reference(golden):
    np.testing.assert_array_equal(otr.badnet_trigger(40, 101, 5), golden["badnet_trigger_101x40"])
    np.testing.assert_array_equal(otr.badnet_trigger(13, 32, 3, 1, 2), golden["badnet_trigger_32x13_s3_d1"])
    mf = np.random.default_rng(0).standard_normal((1, 101, 40)).astype(np.float32)
    ref = mf.copy()
    ref[:, 96:, 35:] = -200
    np.testing.assert_array_equal(otr.add_trigger_to_mfcc(mf, golden["badnet_trigger_101x40"]), ref)


def test_ultrasonic_gate_reproduces_ante_wav(wavs):
    """Known answer: utils/ante.wav == GenerateTrigger(60,'end',cont=True) (ultra_trigger.py:113-120)."""
    trig = wavs["ultrasonic_trigger_int16"].astype(np.float64)[None] / 32768.0
    g = otr.ultrasonic_gate(trig, 60, "end", cont=True)
    ante = wavs["ante_int16"].astype(np.float64) / 32768.0
    np.testing.assert_array_equal(g[0], ante)
    assert np.count_nonzero(wavs["ante_int16"]) == 25509


def test_ultrasonic_noncont_windows(wavs):
    trig = wavs["ultrasonic_trigger_int16"].astype(np.float64)[None] / 32768.0
    g = otr.ultrasonic_gate(trig, 60, "mid", cont=False)
    keep = g[0] != 0
    # 5 windows of int(26460/5) = 5292 samples every 8820
    for k in range(5):
        assert not keep[k * 8820 + 5292:(k + 1) * 8820].any()
    assert np.array_equal(g[0][:5292], trig[0][:5292])
    with pytest.raises(ValueError):
        otr.ultrasonic_gate(trig, 0, "mid")
    with pytest.raises(ValueError):
        otr.ultrasonic_gate(trig, 10, "middle")


def test_cross_entropy_notebook_pin():
    """test.ipynb cell 13: CrossEntropyLoss([[.1,.2,.7],[.8,.1,.1],[.3,.4,.3]], [2,0,1]) = 0.8302483558654785."""
    z = np.array([[.1, .2, .7], [.8, .1, .1], [.3, .4, .3]])
    y = np.array([2, 0, 1])
    lp = oc.log_softmax(z)
    assert -lp[np.arange(3), y].mean() == pytest.approx(0.8302483558654785, rel=1e-7)


def test_mfcc_shapes_notebook_pins():
    """test.ipynb cells 22-27 and attack_config.txt:20-23 frame counts."""
    w = np.random.default_rng(1).standard_normal(16000) * 0.1
    assert om.mfcc_torchaudio(w, 16000, 40, 400, 160).shape == (40, 101)
    assert om.mfcc_torchaudio(w, 16000, 40, 400, 200).shape == (40, 81)
    assert om.mfcc_librosa(w, 16000, 40).shape == (40, 32)
    assert om.mfcc_torchaudio(w[None, None], 16000, 13, 2048, 512).shape == (1, 1, 13, 32)
    w44 = np.random.default_rng(2).standard_normal(44100) * 0.1
    assert om.mfcc_torchaudio(w44, 44100, 40, 1103, 441).shape == (40, 100)


def test_mel_zero_filter_counts_pin():
    """test.ipynb cells 0/22: torchaudio warns of all-zero mel filters; 4/128 at n_fft=400, 1/128 at 1103."""
    fb = om.htk_mel_fbanks(201, 0.0, 8000.0, 128, 16000)
    assert int((fb.max(axis=0) == 0).sum()) == 4
    fb = om.htk_mel_fbanks(552, 0.0, 22050.0, 128, 44100)
    assert int((fb.max(axis=0) == 0).sum()) == 1


def test_stft_stage_matches_torch_stft():
    """The Spectrogram stage torchaudio runs is torch.stft: pin the oracle's STFT against it."""
    import torch
    r = np.random.default_rng(3)
    for L, n_fft, hop in ((16000, 400, 160), (16000, 2048, 512), (44100, 1103, 441)):
        w = (r.standard_normal((2, L)) * 0.2).astype(np.float32)
        t = torch.stft(torch.tensor(w, dtype=torch.float64), n_fft, hop, n_fft, torch.hann_window(n_fft, dtype=torch.float64),
                       center=True, pad_mode="reflect", normalized=False, onesided=True, return_complex=True)
        ref = (t.abs() ** 2).numpy()
        mine = om.stft_power(w, n_fft, hop)
        np.testing.assert_allclose(mine, ref, rtol=1e-9, atol=1e-9 * ref.max())


def test_dct_is_orthonormal():
    d = om.dct_ortho(128, 128)
    np.testing.assert_allclose(d.T @ d, np.eye(128), atol=1e-12)


def test_pydub_semantics():
    host = np.array([1000, -2000, 32000, -32000, 5], dtype=np.int16)
    trig = np.array([100, -100, 1000, -1000], dtype=np.int16)
    out = otr.pydub_overlay(host, trig)
    np.testing.assert_array_equal(out, [1100, -2100, 32767, -32768, 5])
    assert otr.pydub_rms(np.array([3, 4])) == 3  # int(sqrt(12.5)) truncates
    g = otr.pydub_gain(np.array([1000, -1000, 30000], dtype=np.int16), 6.0)
    f = 10 ** (6 / 20)
    np.testing.assert_array_equal(g, [math.floor(1000 * f), math.floor(-1000 * f), 32767])


def test_flowmur_injections_preserve_outside():
    r = np.random.default_rng(4)
    w = r.standard_normal(16000) * 0.1
    t = r.standard_normal(8000) * 0.05
    o = otr.flowmur_train_inject(w, t, 30, 1234)
    np.testing.assert_array_equal(o[:1234], w[:1234])
    d = o[1234:9234] - w[1234:9234]
    snr = 10 * math.log10(np.dot(w, w) / np.dot(d, d))
    assert snr == pytest.approx(30.0, abs=1e-9)
    o2 = otr.flowmur_test_inject(w, t, 10)
    np.testing.assert_allclose(o2[10:8010], (w[10:8010] + t) / 2)


def test_flowmur_oracle_matches_autograd_golden():
    """oracle/flowmur.py's hand-derived adjoints vs torch float64 autograd of the reference loop
    (tests/golden/make_flowmur_golden.py): first-batch gradient and the 2x2 Adam trajectory."""
    import os
    from golden_inputs import FLOWMUR, flowmur_inputs
    from oracle import flowmur as of
    g = dict(np.load(os.path.join(os.path.dirname(__file__), "golden", "flowmur_golden.npz")))
    c = FLOWMUR
    waves, pos, labels, st = flowmur_inputs()
    m = oc.SmallCNN(st)
    B = c["B"]
    loss, dt, feats, out = of.trigger_grad(m, waves[:B].astype(np.float64), np.full(c["Lt"], 0.1), pos[0, 0], labels)
    assert np.abs(feats - g["feats0"]).max() < 1e-10 * np.abs(g["feats0"]).max()
    assert abs(loss - float(g["loss0"])) < 1e-12
    assert np.linalg.norm(dt - g["grad0"]) < 1e-10 * np.linalg.norm(g["grad0"])
    batches = [[(waves[b * B:(b + 1) * B].astype(np.float64), labels, pos[e, b]) for b in range(c["n_batches"])]
               for e in range(c["epochs"])]
    traj = of.optimise(m, batches, c["Lt"], c["epochs"])
    assert np.abs(traj - g["traj"]).max() < 1e-10


# test.ipynb known answers (the notebook's printed outputs; SURVEY §4 items 2 and cells 29-32)
NB12_HEAD, NB12_TAIL = [0.0000, 0.0471, -0.0932], [-0.2744, 0.1865, -0.0942]   # cell 12 (torch 4-digit print)
NB30_HEAD, NB30_TAIL = [-0.00024414, -0.00033569, -0.00033569], [0.00039673, 0.00030518, 0.00048828]  # cell 30
NB29_HEAD, NB29_TAIL = [-0.0002, -0.0003, -0.0003], [0.0004, 0.0003, 0.0005]   # cell 29 (torchaudio.load)
NB32_HEAD, NB32_TAIL = [-16, -22, -22], [26, 20, 32]                             # cell 32: overlay(song, song)


def notebook_test_wav():
    """A 16,000-sample int16 clip whose first and last three samples are test.wav's as printed in
    cell 30 (soundfile float = int16 / 32768: -8, -11, -11 ... 13, 10, 16); test.wav itself is not
    in the reference, so the interior is synthetic -- with saturating samples, which overlay clamps."""
    r = np.random.Generator(np.random.PCG64(30))
    x = r.integers(-20000, 20000, 16000).astype(np.int16)
    x[100:110] = 32767
    x[200:210] = -32768
    x[:3] = np.round(np.array(NB30_HEAD) * 32768).astype(np.int16)
    x[-3:] = np.round(np.array(NB30_TAIL) * 32768).astype(np.int16)
    return x


def test_notebook_cell12_loader_normalisation(wavs):
    """cell 10-12: torchaudio.load(trigger.wav) + torchaudio.load(ante.wav), printed to 4 digits:
    [0.0000, 0.0471, -0.0932, ..., -0.2744, 0.1865, -0.0942] -- int16 / 32768 in float32."""
    from abd_amd import io as aio
    import os
    import tempfile
    s = (wavs["ultrasonic_trigger_int16"].astype(np.float32) / 32768.0
         + wavs["ante_int16"].astype(np.float32) / 32768.0)
    np.testing.assert_array_equal(np.round(s[:3].astype(np.float64), 4), NB12_HEAD)
    np.testing.assert_array_equal(np.round(s[-3:].astype(np.float64), 4), NB12_TAIL)
    # the package's own wav loader (io.read_wav) gives the same sum
    with tempfile.TemporaryDirectory() as d:
        pa, pb = os.path.join(d, "a.wav"), os.path.join(d, "b.wav")
        aio.write_wav_int16(pa, wavs["ultrasonic_trigger_int16"], 44100)
        aio.write_wav_int16(pb, wavs["ante_int16"], 44100)
        (a, sra), (b, srb) = aio.read_wav(pa), aio.read_wav(pb)
    assert sra == srb == 44100 and a.dtype == np.float32
    np.testing.assert_array_equal(a + b, s)


def test_notebook_cells29_32_soundfile_and_overlay():
    """cells 29/30: the clip read by torchaudio (4 decimals) and soundfile (8 decimals);
    cells 31/32: AudioSegment.overlay(song, song) printed as int16 [-16 -22 -22 ... 26 20 32]."""
    x = notebook_test_wav()
    f = x.astype(np.float64) / 32768.0
    np.testing.assert_array_equal(np.round(f[:3], 8), NB30_HEAD)     # numpy's 8-decimal print
    np.testing.assert_array_equal(np.round(f[-3:], 8), NB30_TAIL)
    np.testing.assert_array_equal(np.round(f[:3].astype(np.float32).astype(np.float64), 4), NB29_HEAD)
    np.testing.assert_array_equal(np.round(f[-3:].astype(np.float32).astype(np.float64), 4), NB29_TAIL)
    o = otr.pydub_overlay(x, x)
    np.testing.assert_array_equal(o[:3], NB32_HEAD)
    np.testing.assert_array_equal(o[-3:], NB32_TAIL)
    assert o[105] == 32767 and o[205] == -32768      # saturating add (audioop.add)
    np.testing.assert_array_equal(otr.single_trigger_injection_db(x, x, "keep"), o)
