"""Deterministic inputs/states shared by tests/golden/make_golden.py and the parity tests.

Everything is drawn from numpy PCG64 seeds so the fixtures only need to hold the
reference's OUTPUTS; the tests regenerate the inputs bit-identically.
"""
from __future__ import annotations

import numpy as np

DIGEST_N = 64

# name: (H0, W0, num_classes, linear_features)   -- reference attack_config.txt:11-23
EVAL_CFGS = {
    "jingle101x40": (101, 40, 10, 3072),
    "ultra100x40k35": (100, 40, 35, 3072),
    "daba32x40": (32, 40, 10, 896),
    "flowmur32x13": (32, 13, 10, 224),
}
# name: (H0, W0, K, lf, batch, n_batches)
TRAIN_CFGS = {
    "jingle101x40": (101, 40, 10, 3072, 16, 3),
    "flowmur32x13": (32, 13, 10, 224, 16, 3),
}

PARAM_SHAPES = lambda K, lf: {  # noqa: E731
    "conv1.weight": (64, 1, 2, 2), "conv1.bias": (64,),
    "bn1.weight": (64,), "bn1.bias": (64,),
    "conv2.weight": (64, 64, 2, 2), "conv2.bias": (64,),
    "bn2.weight": (64,), "bn2.bias": (64,),
    "conv3.weight": (32, 64, 2, 2), "conv3.bias": (32,),
    "bn3.weight": (32,), "bn3.bias": (32,),
    "fc1.weight": (128, lf), "fc1.bias": (128,),
    "fc2.weight": (K, 128), "fc2.bias": (K,),
}


def rng(seed):
    return np.random.Generator(np.random.PCG64(seed))


def make_state(H, W, K, lf, seed, trained_bn=False):
    """A smallcnn state_dict (numpy) with torch-like init scales; BN buffers optionally non-trivial."""
    r = rng(seed)
    st = {}
    fan_in = {"conv1": 4, "conv2": 256, "conv3": 256, "fc1": lf, "fc2": 128}
    for k, shp in PARAM_SHAPES(K, lf).items():
        layer = k.split(".")[0]
        if layer.startswith("bn"):
            if k.endswith("weight"):
                v = 1.0 + 0.2 * r.standard_normal(shp)
                v[::7] *= -1.0  # exercise negative gamma (argmax flips to argmin in max-pool)
            else:
                v = 0.1 * r.standard_normal(shp)
        else:
            bound = 1.0 / np.sqrt(fan_in[layer])
            v = r.uniform(-bound, bound, shp)
        st[k] = v.astype(np.float32)
    for i, c in ((1, 64), (2, 64), (3, 32)):
        if trained_bn:
            st[f"bn{i}.running_mean"] = (r.standard_normal(c) * 0.5 + 0.5).astype(np.float32)
            st[f"bn{i}.running_var"] = (r.uniform(0.2, 3.0, c)).astype(np.float32)
        else:
            st[f"bn{i}.running_mean"] = np.zeros(c, np.float32)
            st[f"bn{i}.running_var"] = np.ones(c, np.float32)
        st[f"bn{i}.num_batches_tracked"] = np.array(0, dtype=np.int64)
    return st


def mfcc_like(r, n, H, W):
    """Plausible MFCC magnitudes: c0 strongly negative, higher coefficients shrinking."""
    x = r.standard_normal((n, 1, H, W)) * (20.0 / (1.0 + np.arange(W) / 8.0))
    x[..., 0] = -250.0 + 40.0 * r.standard_normal((n, 1, H))
    return x.astype(np.float32)


def patch(x, s=5):
    """BadNets -200 square on the last s frames x last s coefficients (utils/badnet_trigger.py:4-27)."""
    x[..., -s:, -s:] = -200.0
    return x


def eval_inputs(H, W, n=4):
    r = rng(31 + H + W)
    x = mfcc_like(r, n, H, W)
    patch(x[1:2])
    return x


def train_inputs(H, W, K, B, NB):
    r = rng(77 + H + W + K)
    N = B * NB
    x = mfcc_like(r, N, H, W)
    y = r.integers(0, K, N).astype(np.int64)
    ind = (r.random(N) < 0.3).astype(np.int64)
    ind[0] = 1
    for i in np.nonzero(ind)[0]:
        patch(x[i:i + 1])
        y[i] = 2
    xc = mfcc_like(r, 2 * B, H, W)
    yc = r.integers(0, K, 2 * B).astype(np.int64)
    xb = mfcc_like(r, 2 * B, H, W)
    ib = (r.random(2 * B) < 0.8).astype(np.int64)
    for i in np.nonzero(ib)[0]:
        patch(xb[i:i + 1])
    yb = np.full(2 * B, 2, dtype=np.int64)
    return x, y, ind, xc, yc, xb, yb, ib


FLOWMUR = dict(B=4, L=16000, Lt=8000, n_batches=2, epochs=2, K=10, H=32, W=13, lf=224)


def flowmur_inputs(seed=91):
    """FlowMur trigger-optimisation fixture inputs: int16-quantised 1 s clips (two tones + noise),
    all labelled 2 (flowmur_generate_trigger.py:143), window positions per (epoch, batch, row)."""
    c = FLOWMUR
    r = rng(seed)
    t = np.arange(c["L"]) / 16000.0
    n = c["B"] * c["n_batches"]
    waves = np.empty((n, c["L"]), np.float32)
    for i in range(n):
        f1, f2 = r.uniform(150.0, 3500.0, 2)
        w = 0.3 * np.sin(2 * np.pi * f1 * t + r.uniform(0, 2 * np.pi)) + 0.2 * np.sin(2 * np.pi * f2 * t) * \
            (0.5 + 0.5 * np.sin(2 * np.pi * r.uniform(2, 8) * t)) + 0.05 * r.standard_normal(c["L"])
        waves[i] = np.round(np.clip(w, -1, 1) * 32767) / 32768.0
    pos = r.integers(0, c["L"] - c["Lt"] + 1, (c["epochs"], c["n_batches"], c["B"]))
    labels = np.full(c["B"], 2, np.int64)
    state = make_state(c["H"], c["W"], c["K"], c["lf"], seed=seed + 1, trained_bn=True)
    return waves, pos, labels, state


# Multi-epoch convergence fixtures (tests/golden/make_convergence.py): the reference's own
# eval_model loop (badnets.py:127-160 / ultrasonic.py:155-188: model built, fix_random(), poisoned
# data, shuffled loaders, train() + test() per epoch) on synthetic class-conditional clips.
CONV_CFGS = {
    "badnets": dict(attack="badnets", sr=16000, L=16000, n_fft=400, hop=160, n_mfcc=40, K=10, lf=3072, B=256,
                    n_train=2048, n_test=512, epochs=8, clip_seed=101, init_seed=1234),
    "ultrasonic": dict(attack="ultrasonic", sr=44100, L=44100, n_fft=1103, hop=441, n_mfcc=40, K=35, lf=3072,
                       B=512, n_train=4096, n_test=1024, epochs=14, clip_seed=102, init_seed=1235),
    # jingleback.py:127-197 (style 5 board, B = 256 hard-coded at :129-132), daba.py:142-219
    # (librosa MFCC 32 x 40, fc 896, args.batch_size 256), flowmur.py:42-191 (clean-label, MFCC
    # 2048/512 with 13 coefficients -> 32 x 13, fc 224, args.batch_size 256)
    "jingleback": dict(attack="jingleback", sr=16000, L=16000, n_fft=400, hop=160, n_mfcc=40, K=10, lf=3072, B=256,
                       n_train=2048, n_test=512, epochs=8, clip_seed=103, init_seed=1236),
    "daba": dict(attack="daba", sr=16000, L=16000, n_fft=2048, hop=512, n_mfcc=40, K=10, lf=896, B=256,
                 n_train=4096, n_test=1024, epochs=12, clip_seed=104, init_seed=1237),
    "flowmur": dict(attack="flowmur", sr=16000, L=16000, n_fft=2048, hop=512, n_mfcc=13, K=10, lf=224, B=256,
                    n_train=4096, n_test=1024, epochs=12, clip_seed=105, init_seed=1238, snr_db=30, Lt=8000),
}


def ultrasonic_trigger_f32():
    """GenerateTrigger(60, 'mid', cont=False).trigger() (ultrasonic.py:41-42 defaults, utils/ultra_trigger.py)
    on the packaged trigger.wav samples, as float32 (torchaudio.load's dtype)."""
    import os
    from oracle.triggers import ultrasonic_gate
    here = os.path.dirname(os.path.abspath(__file__))
    t = np.load(os.path.join(here, "golden", "ultrasonic_wavs.npz"))["ultrasonic_trigger_int16"]
    return ultrasonic_gate(t[None].astype(np.float64) / 32768.0, 60, "mid", cont=False).astype(np.float32)


def daba_trigger_int16():
    """resources/DABA/trigger_pool/music0_0.wav (the fixture copy in daba_golden.npz)."""
    import os
    here = os.path.dirname(os.path.abspath(__file__))
    return np.load(os.path.join(here, "golden", "daba_golden.npz"))["pool0"].copy()


def flowmur_trigger_f32(Lt=8000):
    """The optimised trigger of the flowmur fixture, in place of sp_trigger300.npy (flowmur.py:67,
    not in the reference): made by tests/golden/make_flowmur_conv_trigger.py the way the
    reference's generate_trigger would (surrogate smallcnn + SNR-30 mix + MFCC + CE to label 2)."""
    import os
    here = os.path.dirname(os.path.abspath(__file__))
    t = np.load(os.path.join(here, "golden", "flowmur_conv_trigger.npy"))
    assert t.shape == (Lt,) and t.dtype == np.float32
    return t


def convergence_data(name):
    """Clean / poisoned features exactly as the attack's poisoning step builds them, from
    deterministic synthetic clips: badnets_poison_data (badnets.py:38-95), ultrasonic_poison_data
    (ultrasonic.py:40-124), style_poison_data (jingleback.py:38-119, style 5), daba_poison_data's
    injection + get_data (utils/daba_injection_tools.py:102-211, daba.py:55-82) and
    flowmur_poison_data (flowmur.py:42-127).

    Must run right after fix_random() (it draws the poisoned rows with the global ``random`` /
    ``np.random``).  torchaudio features come from oracle.torch_ref.mfcc (the torch-CPU restatement
    of T.MFCC), librosa's from oracle.mfcc.mfcc_librosa (float64, then ``.float()``), the style board
    from oracle.effects.style5, pydub's overlay from oracle.triggers.
    DABA's trigger / host SELECTION (certainty + influence, daba_selection_tools.py:154-160) is not
    replayed here: its inputs are an untrained model's batch-1 forwards, pinned separately
    (tests/golden/daba_golden.npz); the hosts are a random.sample of the non-target train clips and
    the trigger is the pool's first clip, with the reference's variant-dB schedule."""
    import random

    import torch
    from abd_amd import synth
    from oracle import torch_ref
    c = CONV_CFGS[name]
    if c["attack"] == "daba":
        return _daba_convergence_data(c)
    if c["attack"] == "flowmur":
        return _flowmur_convergence_data(c)
    n = c["n_train"] + c["n_test"]
    waves, labels = synth.make_clips_np(n, c["sr"], c["L"], c["K"], seed=c["clip_seed"])

    def feats(w):
        return torch_ref.mfcc(torch.from_numpy(np.ascontiguousarray(w)), c["sr"], c["n_mfcc"], c["n_fft"],
                              c["hop"]).numpy()

    clean = feats(waves)
    ntr = c["n_train"]
    tr_x, te_x = clean[:ntr].copy(), clean[ntr:].copy()
    tr_y, te_y = labels[:ntr].copy(), labels[ntr:].copy()
    T, C = tr_x.shape[2], tr_x.shape[3]
    rows = random.sample(list(range(ntr)), int(ntr * 0.1))      # badnets.py:50-51 / ultrasonic.py:70-71
    ind = np.zeros(ntr, np.int64)
    ind[rows] = 1
    bd_y = tr_y.copy()
    bd_y[rows] = 2
    test_pois = te_y != 2
    if c["attack"] == "badnets":
        def poison(x):
            x[:, :, T - 5:T, C - 5:C] = -200.0   # generate_trigger(W, H, 5) + add_trigger_to_mfcc
            return x
        bd_x = tr_x.copy()
        bd_x[rows] = poison(bd_x[rows])
        bt_x = te_x.copy()
        bt_x[test_pois] = poison(bt_x[test_pois])
    elif c["attack"] == "jingleback":
        from oracle import effects as oe

        def styled(w):   # pedalboard runs float32 (styles_trigger.py:51-53)
            return oe.style5(w, c["sr"]).astype(np.float32)
        bd_x = tr_x.copy()
        srt = np.sort(rows)
        bd_x[srt] = feats(styled(waves[:ntr][srt]))
        bt_x = te_x.copy()
        bt_x[test_pois] = feats(styled(waves[ntr:][test_pois]))
    else:
        trig = ultrasonic_trigger_f32()
        bd_x = tr_x.copy()
        srt = np.sort(rows)
        bd_x[srt] = feats(waves[:ntr][srt] + trig)
        bt_x = te_x.copy()
        bt_x[test_pois] = feats(waves[ntr:][test_pois] + trig)
    return dict(bd_x=bd_x, bd_y=bd_y.astype(np.int64), ind=ind, clean_x=te_x, clean_y=te_y.astype(np.int64),
                bt_x=bt_x, bt_y=np.full(c["n_test"], 2, np.int64), bt_ind=test_pois.astype(np.int64))


def _daba_convergence_data(c):
    import random

    from abd_amd import synth
    from oracle import mfcc as om
    from oracle import triggers as otr
    n = c["n_train"] + c["n_test"]
    waves, labels = synth.make_clips_np(n, c["sr"], c["L"], c["K"], seed=c["clip_seed"])
    pcm = np.round(waves.astype(np.float64) * 32768.0).astype(np.int16)       # the wav files' samples
    ntr, target = c["n_train"], 2                                              # 'up' = SCDv1-10 index 2
    tr_y, te_y = labels[:ntr].copy(), labels[ntr:].copy()
    hosts = [i for i in range(ntr) if tr_y[i] != target]
    poison_num = round(c.get("rate", 0.1) * ntr)                               # daba_injection_tools.py:116-117
    rows = sorted(random.sample(hosts, poison_num))
    mean_db = otr.gen_trigger_variants_db(poison_num)                          # :136-137 (re-seeds random)
    trig = daba_trigger_int16()

    def feats(p16):   # soundfile -> librosa_MFCC(.., 40).T[np.newaxis] -> torch.tensor(..).float()
        w = np.asarray(p16).astype(np.float64) / 32768.0       # (== om.mfcc_librosa per clip, batched)
        out = [om.mfcc_core(w[s:s + 256], c["sr"], c["n_mfcc"], c["n_fft"], c["hop"], mel="slaney",
                            pad_mode="constant") for s in range(0, len(w), 256)]
        return np.transpose(np.concatenate(out), (0, 2, 1))[:, None].astype(np.float32)

    tr_x, te_x = feats(pcm[:ntr]), feats(pcm[ntr:])
    bd_x, bd_y = tr_x.copy(), tr_y.copy()
    ind = np.zeros(ntr, np.int64)
    bd_x[rows] = feats([otr.single_trigger_injection_db(pcm[r], trig, mean_db[k]) for k, r in enumerate(rows)])
    bd_y[rows] = target
    ind[rows] = 1
    test_pois = te_y != target                                                 # :203-209 (po_db = -20)
    bt_x = te_x.copy()
    bt_x[test_pois] = feats([otr.single_trigger_injection_db(pcm[ntr + i], trig, -20)
                             for i in np.nonzero(test_pois)[0]])
    return dict(bd_x=bd_x, bd_y=bd_y.astype(np.int64), ind=ind, clean_x=te_x, clean_y=te_y.astype(np.int64),
                bt_x=bt_x, bt_y=np.full(c["n_test"], target, np.int64), bt_ind=test_pois.astype(np.int64))


def _flowmur_convergence_data(c):
    import random

    import torch
    from abd_amd import synth
    from oracle import torch_ref
    n = c["n_train"] + c["n_test"]
    waves, labels = synth.make_clips_np(n, c["sr"], c["L"], c["K"], seed=c["clip_seed"])
    ntr, target, Lt = c["n_train"], 2, c["Lt"]
    trw = torch.from_numpy(waves[:ntr].copy())[:, None]       # (N, 1, L) float32 like the reference
    tew = torch.from_numpy(waves[ntr:].copy())[:, None]
    tr_y, te_y = labels[:ntr].copy(), labels[ntr:].copy()
    trigger = torch.from_numpy(flowmur_trigger_f32(Lt))[None]
    tidx = np.where(tr_y == target)[0]                        # flowmur.py:74-76
    poison_num = int(tidx.shape[0] * 0.1)
    pidx = np.random.choice(tidx, poison_num, replace=False)
    trigger_rms = torch.linalg.norm(trigger.clone(), dim=1)
    for i in pidx:                                            # :78-85
        wav_rms = torch.linalg.norm(trw[i].clone(), dim=1)
        scale = torch.sqrt(torch.pow(wav_rms, 2) / torch.pow(trigger_rms, 2) * (10 ** (-c["snr_db"] / 10)))
        pos = random.randint(0, trw.shape[2] - Lt)
        trw[i][0][pos:pos + Lt] = trw[i][0][pos:pos + Lt] + scale * trigger[0]

    def feats(w):     # MFCC(...).permute(0, 1, 3, 2) -> (N, 1, T, 13)
        return torch_ref.mfcc(w[:, 0].contiguous(), c["sr"], c["n_mfcc"], c["n_fft"], c["hop"]).numpy()

    bd_x = feats(trw)
    ind = (tr_y == target).astype(np.int64)                   # :88-89 (every target clip counts)
    clean_x = feats(tew)                                      # :93
    keep = np.where(te_y != target)[0]                        # :95-99
    bw = tew[keep].clone()
    for i in range(bw.shape[0]):                              # :100-105
        pos = random.randint(0, bw.shape[2] - Lt)
        bw[i][0] = torch.cat([bw[i][0][:pos] / 2, (bw[i][0][pos:pos + Lt] + trigger[0]) / 2, bw[i][0][pos + Lt:] / 2])
    bt_x = feats(bw)
    return dict(bd_x=bd_x, bd_y=tr_y.astype(np.int64), ind=ind, clean_x=clean_x, clean_y=te_y.astype(np.int64),
                bt_x=bt_x, bt_y=np.full(len(keep), target, np.int64), bt_ind=np.ones(len(keep), np.int64))


def data_digest(d):
    return np.array([float(np.asarray(d[k], np.float64).sum()) for k in sorted(d)] +
                    [float(np.abs(np.asarray(d[k], np.float64)).sum()) for k in sorted(d)])


def unpack_mask(packed, n_cols):
    return np.unpackbits(packed, axis=-1)[..., :n_cols].astype(np.float64)
