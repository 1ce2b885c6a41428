"""GPU: the drop-in modules driven the way the attack scripts drive them.

* ``prepare_clean_dataset`` / ``load_clean_data`` (prepare_dataset.py:49-112) on a synthetic
  Speech-Commands tree: kept clips, labels, the 80/20 split (random_state 35) and the MFCC cache
  match a restatement (stdlib wav read, float64 oracle MFCC, sklearn split); the 16 -> 44.1 kHz
  resampling path (ultrasonic) likewise against the oracle resampler.
* an eval_model-shaped script (badnets.py:127-175 restated: poison, loaders, train() + test() +
  EarlyStoppingModel per epoch) run with ``python -m abd_amd.run`` -- every import through the
  drop-in -- and the whole-module ``checkpoint.pt`` it writes (training_tools.py:44-50) reloaded:
  identical state_dict and identical eval log-probs.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

import abd_amd
from abd_amd import synth
from abd_amd.io import LABEL_SETS, write_wav_int16
from oracle import mfcc as om

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DROPIN = os.path.join(ROOT, "audio-backdoor-attack_amd", "dropin")


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    abd_amd.load_library()
    return torch.device("cuda", 0)


def write_tree(root, labels, per_label=12, sr=16000, seed=3):
    """Clips per label dir; every 5th clip is 0.75 s long (prepare_dataset.py:61 drops it)."""
    w, _ = synth.make_clips_np(len(labels) * per_label, sr, sr, len(labels), seed=seed)
    i = 0
    for li, lab in enumerate(labels):
        d = os.path.join(root, lab)
        os.makedirs(d, exist_ok=True)
        for k in range(per_label):
            clip = w[i] if k % 5 else w[i][: 3 * sr // 4]
            # class-dependent content: scale the clip by the label so labels are learnable
            q = np.clip(np.round(clip * (0.3 + 0.07 * li) * 32768.0), -32768, 32767).astype(np.int16)
            write_wav_int16(os.path.join(d, f"clip{k:03d}.wav"), q, sr)
            i += 1


def restated_clean(data_path, labels, sr, n_mfcc, n_fft, hop):
    """prepare_dataset.py:49-84 restated with the stdlib reader and the float64 oracle."""
    from abd_amd.io import read_wav
    from sklearn.model_selection import train_test_split
    waves, labs = [], []
    for li, lab in enumerate(labels):
        d = os.path.join(data_path, lab)
        for name in os.listdir(d):
            if name.endswith(".wav"):
                w, rate = read_wav(os.path.join(d, name))
                if rate != sr:
                    from oracle import resample as ors
                    w = ors.resample(w.astype(np.float64), rate, sr).astype(np.float32)
                if w.shape[0] >= sr:
                    waves.append(w[None])
                    labs.append(li)
    mf = [om.mfcc_model_input(x.astype(np.float64), sr, n_mfcc, n_fft, hop)[0] for x in waves]
    return train_test_split(waves, mf, labs, test_size=0.2, random_state=35)


@pytest.mark.parametrize("sr,n_fft,hop", [(16000, 400, 160), (44100, 1103, 441)])
def test_prepare_clean_dataset_matches_restatement(dev, tmp_path, sr, n_fft, hop):
    sys.path.insert(0, DROPIN)
    try:
        import prepare_dataset as pd   # the drop-in module
    finally:
        sys.path.remove(DROPIN)
    labels = ["yes", "no", "up"]
    data = tmp_path / "data"
    write_tree(str(data), labels, per_label=6, sr=16000)
    out = pd.prepare_clean_dataset(str(data), str(tmp_path / "rec"), labels, sr, 40, n_fft, hop, sr=sr, save=True)
    ref = restated_clean(str(data), labels, sr, 40, n_fft, hop)
    tr_w, te_w, tr_m, te_m, tr_y, te_y = out
    assert tr_w.shape == (len(ref[0]), 1, sr) and te_w.shape == (len(ref[1]), 1, sr)
    assert np.array_equal(tr_y, np.array(ref[4])) and np.array_equal(te_y, np.array(ref[5]))
    tol = 0.0 if sr == 16000 else 3e-6   # the resampled path: float32 device FIR vs float64 restatement
    assert np.abs(tr_w - np.array(ref[0])).max() <= tol and np.abs(te_w - np.array(ref[1])).max() <= tol
    for mine, r in ((tr_m, np.array(ref[2])), (te_m, np.array(ref[3]))):
        err = np.abs(mine - r).reshape(len(r), -1).max(1) / np.abs(r).reshape(len(r), -1).max(1)
        assert err.max() < 1e-4, err.max()
    # the .npy cache prepare_dataset.py:74-83 writes, read back by load_clean_data(load=True)
    cached = np.load(str(tmp_path / "rec" / "clean" / "clean_train_mfcc.npy"))
    assert np.array_equal(cached, tr_m)


SCRIPT = r'''
import json, os, random, sys
import numpy as np
import torch, torch.nn as nn, torch.optim as optim, torch.utils.data as Data
from prepare_dataset import MFCC, load_clean_data, BDDataset
from utils.random_tools import fix_random
from utils.badnet_trigger import add_trigger_to_mfcc, generate_trigger
from utils.training_tools import train, test, EarlyStoppingModel
from utils.models import smallcnn

class Args:   # badnets.py:17-36 defaults (smallcnn, SCDv1-10), 3 epochs
    model, dataset, result = "smallcnn", "SCDv1-10", "badnets_smallcnn"
    sample_rate, n_mfcc, n_fft, hop_length, trigger_size, poisoning_rate = 16000, 40, 400, 160, 5, 0.1
    learning_rate, num_epochs, patience = 1e-4, 3, 20
args = Args()

def badnets_poison_data(train_wav, test_wav, train_mfcc, test_mfcc, train_label, test_label):
    """badnets.py:38-95 (poisoning restated; the imports are the drop-in's)"""
    trigger = generate_trigger(test_mfcc[0].shape[2], test_mfcc[0].shape[1], args.trigger_size, save=False)
    poison = random.sample(list(range(len(train_wav))), int(len(train_wav) * args.poisoning_rate))
    bx, by, bi = [], [], []
    for i in range(len(train_wav)):
        if i in poison:
            bx.append(add_trigger_to_mfcc(train_mfcc[i], trigger)); by.append(2); bi.append(1)
        else:
            bx.append(train_mfcc[i]); by.append(train_label[i]); bi.append(0)
    tx, ty, ti = [], [], []
    for i in range(len(test_wav)):
        if test_label[i] == 2:
            tx.append(test_mfcc[i]); ti.append(0)
        else:
            m = MFCC(torch.tensor(test_wav[i].squeeze(0)), args.sample_rate, args.n_mfcc, args.n_fft,
                     args.hop_length).numpy().T[np.newaxis, :]
            tx.append(add_trigger_to_mfcc(m, trigger)); ti.append(1)
        ty.append(2)
    return (np.array(bx), np.array(tx), np.array(by), np.array(ty), np.array(bi), np.array(ti))

model = smallcnn(10, 3072)
device = torch.device("cuda")
model.to(device)
criterion = nn.CrossEntropyLoss()
optimizer = optim.Adam(model.parameters(), lr=args.learning_rate)
fix_random()
data_path = "record/" + args.result
clean = load_clean_data(args=args, load=False)
bx, tx, by, ty, bi, ti = badnets_poison_data(*clean)
clean_test_loader = Data.DataLoader(Data.TensorDataset(torch.tensor(clean[3]), torch.tensor(clean[5])),
                                    batch_size=256, shuffle=True)
bd_train_loader = Data.DataLoader(BDDataset(torch.tensor(bx), torch.tensor(by), torch.tensor(bi)),
                                  batch_size=256, shuffle=True)
bd_test_loader = Data.DataLoader(BDDataset(torch.tensor(tx), torch.tensor(ty), torch.tensor(ti)),
                                 batch_size=256, shuffle=True)
early_stopping = EarlyStoppingModel(patience=args.patience, verbose=True, path=data_path + "/checkpoint.pt")
hist = []
for epoch in range(1, args.num_epochs + 1):
    tr = train(model=model, train_loader=bd_train_loader, device=device, optimizer=optimizer, criterion=criterion)
    te = test(model=model, device=device, clean_test_loader=clean_test_loader, bd_test_loader=bd_test_loader,
              criterion=criterion)
    early_stopping(0.5 * (te[2] + te[3]), model=model)
    hist.append([*tr, *te])
# whole-module checkpoint round trip (utils/training_tools.py:49 torch.save(model, path))
torch.save(model, "roundtrip.pt")
m2 = torch.load("roundtrip.pt", map_location=device, weights_only=False)
sd1, sd2 = model.state_dict(), m2.state_dict()
same_sd = sorted(sd1) == sorted(sd2) and all(torch.equal(sd1[k].cpu(), sd2[k].cpu()) for k in sd1)
x = torch.tensor(tx[:16]).to(device)
model.eval(); m2.eval()
with torch.no_grad():
    same_out = bool(torch.equal(model(x), m2(x)))
torch.save({k: v.cpu() for k, v in sd1.items()}, "final_state_dict.pt")
json.dump({"hist": hist, "same_sd": same_sd, "same_out": same_out, "n_train": len(bx), "n_test": len(tx),
           "n_poison": int(bi.sum()), "modules": {n: sys.modules[n].__file__ for n in
           ("prepare_dataset", "utils.training_tools", "utils.models")}}, open(sys.argv[1], "w"))
'''


def test_eval_model_loop_through_dropins_and_checkpoint(dev, tmp_path):
    path, labels = LABEL_SETS["SCDv1-10"]
    write_tree(str(tmp_path / path), labels, per_label=30)
    (tmp_path / "badnets_like.py").write_text(SCRIPT)
    out = tmp_path / "res.json"
    env = dict(os.environ, PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-m", "abd_amd.run", "badnets_like.py", str(out)], cwd=tmp_path, env=env,
                       capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-4000:]
    res = json.loads(out.read_text())
    assert all("dropin" in f for f in res["modules"].values()), res["modules"]
    assert res["same_sd"] and res["same_out"]
    h = np.array(res["hist"])                       # train loss, mix acc, train asr, clean acc, asr, losses
    assert np.all(np.isfinite(h)) and h[-1, 0] < h[0, 0]
    assert res["n_poison"] == int(res["n_train"] * 0.1)
    # the early-stopping checkpoint loads in another process and runs
    from conftest import load_dropin_checkpoint
    ck = load_dropin_checkpoint(str(tmp_path / "record" / "badnets_smallcnn" / "checkpoint.pt"), map_location=dev)
    ck.eval()
    with torch.no_grad():
        y = ck(torch.zeros((2, 1, 101, 40), device=dev))
    assert y.shape == (2, 10) and torch.isfinite(y).all()
    # the state_dict is the reference's layout (keys / shapes of utils/models.py smallcnn)
    sd = torch.load(str(tmp_path / "final_state_dict.pt"), weights_only=True)
    from oracle import torch_ref
    ref = torch_ref.SmallCNN(10, 3072)
    ref.load_state_dict(sd, strict=True)
