#!/usr/bin/env python3
"""Generate golden vectors by importing the REFERENCE's own Python modules.

Run in the build container (where /root/reference exists):
    python tests/golden/make_golden.py
Outputs small .npz fixtures next to this script.  Nothing from the reference is
copied: inputs are generated here from numpy PCG64 seeds (so tests can regenerate
them), the reference code is executed, and only its outputs are stored.

Reference modules exercised (importable here without torchaudio/librosa/pydub):
  utils/models.py            smallcnn (eval logits; train-mode forward/backward)
  utils/training_tools.py    train() (:52-85) and test() (:87-134) with torch Adam
  utils/badnet_trigger.py    generate_trigger (:4-16)
and the data files resources/Ultrasonic/trigger.wav + utils/ante.wav (read with
the stdlib ``wave`` module) for the Ultrasonic known answer.
"""
from __future__ import annotations

import os
import sys
import wave

import numpy as np

REF = os.environ.get("ABD_REFERENCE", "/root/reference")
HERE = os.path.dirname(os.path.abspath(__file__))
sys.dont_write_bytecode = True
sys.path.insert(0, REF)
sys.path.insert(0, os.path.dirname(HERE))  # tests/ for golden_inputs

import torch  # noqa: E402

from golden_inputs import (EVAL_CFGS, TRAIN_CFGS, eval_inputs, make_state,  # noqa: E402
                           train_inputs, DIGEST_N)

import utils.models as ref_models  # noqa: E402
import utils.training_tools as ref_tt  # noqa: E402
import utils.badnet_trigger as ref_bt  # noqa: E402


class DictSet(torch.utils.data.Dataset):
    """Same item contract as the reference BDDataset (prepare_dataset.py:13-33)."""

    def __init__(self, x, y, ind):
        self.x, self.y, self.ind = x, y, ind

    def __len__(self):
        return len(self.x)

    def __getitem__(self, i):
        return {"mfcc": self.x[i], "label": self.y[i], "poison_indicator": self.ind[i]}


def to_torch_state(model, state):
    sd = {k: torch.tensor(v) for k, v in state.items()}
    model.load_state_dict(sd)


def digest(t: np.ndarray, seed: int):
    t = np.asarray(t, dtype=np.float64).reshape(-1)
    rng = np.random.Generator(np.random.PCG64(seed))
    idx = rng.choice(t.size, size=min(DIGEST_N, t.size), replace=False)
    return np.concatenate([[t.sum(), np.sqrt((t * t).sum())], t[idx]])


def gen_eval(out):
    for name, (H, W, K, lf) in EVAL_CFGS.items():
        state = make_state(H, W, K, lf, seed=1000 + H * 7 + W + K, trained_bn=True)
        m = ref_models.smallcnn(K, lf)
        to_torch_state(m, state)
        m.eval()
        x = eval_inputs(H, W)
        with torch.no_grad():
            y = m(torch.tensor(x)).numpy()
        out[f"eval_{name}_logprobs"] = y


def gen_train(out):
    for name, (H, W, K, lf, B, NB) in TRAIN_CFGS.items():
        state = make_state(H, W, K, lf, seed=2000 + H * 7 + W + K, trained_bn=False)
        m = ref_models.smallcnn(K, lf)
        to_torch_state(m, state)
        x, y, ind, xc, yc, xb, yb, ib = train_inputs(H, W, K, B, NB)

        masks = {"drop1": [], "drop2": []}
        outs = []

        def mk(nm):
            def hook(mod, inp, o):
                if mod.training:
                    keep = (o.detach() != 0) | (inp[0].detach() == 0)
                    masks[nm].append(np.packbits(keep.numpy().reshape(keep.shape[0], -1).astype(np.uint8), axis=-1))
            return hook

        m.drop1.register_forward_hook(mk("drop1"))
        m.drop2.register_forward_hook(mk("drop2"))
        m.register_forward_hook(lambda mod, i, o: outs.append(o.detach().numpy().copy()) if mod.training else None)
        grads0 = {}
        hooks = []
        for pn, p in m.named_parameters():
            def ghook(g, pn=pn):
                grads0.setdefault(pn, g.detach().numpy().copy())
            hooks.append(p.register_hook(ghook))

        torch.manual_seed(7)
        opt = torch.optim.Adam(m.parameters(), lr=1e-4)
        crit = torch.nn.CrossEntropyLoss()
        loader = torch.utils.data.DataLoader(DictSet(torch.tensor(x), torch.tensor(y), torch.tensor(ind)),
                                             batch_size=B, shuffle=False)
        tr = ref_tt.train(m, loader, torch.device("cpu"), opt, crit)
        for h in hooks:
            h.remove()
        clean = torch.utils.data.DataLoader(torch.utils.data.TensorDataset(torch.tensor(xc), torch.tensor(yc)),
                                            batch_size=B, shuffle=False)
        bd = torch.utils.data.DataLoader(DictSet(torch.tensor(xb), torch.tensor(yb), torch.tensor(ib)),
                                         batch_size=B, shuffle=False)
        te = ref_tt.test(m, torch.device("cpu"), clean, bd, crit)

        out[f"train_{name}_result"] = np.array(tr, dtype=np.float64)
        out[f"test_{name}_result"] = np.array(te, dtype=np.float64)
        out[f"train_{name}_mask1"] = np.stack(masks["drop1"])
        out[f"train_{name}_mask2"] = np.stack(masks["drop2"])
        out[f"train_{name}_outs"] = np.stack(outs)
        sd = {k: v.detach().numpy() for k, v in m.state_dict().items()}
        pid = {p: n for n, p in m.named_parameters()}
        for k, v in sd.items():
            out[f"train_{name}_final_{k}"] = digest(v, 11)
        for k, v in grads0.items():
            out[f"train_{name}_grad0_{k}"] = digest(v, 12)
        for p, st in opt.state.items():
            out[f"train_{name}_expavg_{pid[p]}"] = digest(st["exp_avg"].numpy(), 13)
            out[f"train_{name}_expavgsq_{pid[p]}"] = digest(st["exp_avg_sq"].numpy(), 14)


def gen_init(out):
    """Reference smallcnn default init under a fixed torch seed (the drop-in must match it)."""
    for K, lf in ((10, 3072), (35, 3072), (10, 224)):
        torch.manual_seed(123)
        m = ref_models.smallcnn(K, lf)
        for k, v in m.state_dict().items():
            out[f"init_{K}_{lf}_{k}"] = digest(v.numpy(), 15)


def gen_badnets(out):
    out["badnet_trigger_101x40"] = ref_bt.generate_trigger(40, 101, 5, save=False)
    out["badnet_trigger_32x13_s3_d1"] = ref_bt.generate_trigger(13, 32, 3, 1, 2, save=False)


def read_wav_int16(path):
    with wave.open(path) as w:
        assert w.getsampwidth() == 2 and w.getnchannels() == 1
        return np.frombuffer(w.readframes(w.getnframes()), dtype=np.int16).copy(), w.getframerate()


def gen_wavs(out):
    trig, sr = read_wav_int16(os.path.join(REF, "resources/Ultrasonic/trigger.wav"))
    ante, sr2 = read_wav_int16(os.path.join(REF, "utils/ante.wav"))
    assert sr == sr2 == 44100
    out["ultrasonic_trigger_int16"] = trig
    out["ante_int16"] = ante
    return trig


def main():
    torch.set_num_threads(4)
    out = {}
    gen_eval(out)
    gen_train(out)
    gen_init(out)
    gen_badnets(out)
    np.savez_compressed(os.path.join(HERE, "golden_ref.npz"), **out)
    wavs = {}
    trig = gen_wavs(wavs)
    np.savez_compressed(os.path.join(HERE, "ultrasonic_wavs.npz"), **wavs)
    res = os.path.join(os.path.dirname(os.path.dirname(HERE)), "audio-backdoor-attack_amd", "resources")
    os.makedirs(res, exist_ok=True)
    np.save(os.path.join(res, "ultrasonic_trigger_int16.npy"), trig)
    print("wrote", sorted(out)[:6], "...", len(out), "arrays")


if __name__ == "__main__":
    main()
