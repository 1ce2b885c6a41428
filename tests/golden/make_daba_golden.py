#!/usr/bin/env python3
"""Golden vectors for DABA selection: the REFERENCE's smallcnn (utils/models.py) run the way
utils/daba_selection_tools.py:68-87 runs it -- a fresh model (train mode) forwarded on ONE
clip at a time -- with the dropout masks captured by hooks, plus a few trigger-pool clips.

    python tests/golden/make_daba_golden.py      (in the build container, /root/reference present)

Inputs are generated here (numpy PCG64) except the pool clips, which are data files of the
reference (resources/DABA/trigger_pool/*.wav, read with the stdlib ``wave`` module)."""
from __future__ import annotations

import glob
import os
import sys
import wave

import numpy as np

REF = os.environ.get("ABD_REFERENCE", "/root/reference")
HERE = os.path.dirname(os.path.abspath(__file__))
sys.dont_write_bytecode = True
sys.path.insert(0, REF)
sys.path.insert(0, os.path.dirname(HERE))

import torch  # noqa: E402

from golden_inputs import make_state, mfcc_like  # noqa: E402
import utils.models as ref_models  # noqa: E402

H, W, K, LF = 32, 40, 10, 896
N = 6


def main():
    torch.set_num_threads(4)
    out = {}
    state = make_state(H, W, K, LF, seed=4321, trained_bn=False)
    m = ref_models.smallcnn(K, LF)
    m.load_state_dict({k: torch.tensor(v) for k, v in state.items()})
    r = np.random.Generator(np.random.PCG64(77))
    x = mfcc_like(r, N, H, W).astype(np.float32)
    x[1, 0, 25:, :] = -200.0   # a short clip's padded tail (daba_selection_tools.py:75)
    masks = {"drop1": [], "drop2": []}

    def mk(nm):
        def hook(mod, inp, o):
            keep = (o.detach() != 0) | (inp[0].detach() == 0)
            masks[nm].append(np.packbits(keep.numpy().reshape(keep.shape[0], -1).astype(np.uint8), axis=-1))
        return hook

    m.drop1.register_forward_hook(mk("drop1"))
    m.drop2.register_forward_hook(mk("drop2"))
    torch.manual_seed(35)
    lps = []
    for i in range(N):                       # one batch-1 train-mode forward per clip
        with torch.no_grad():
            lps.append(m.forward(torch.tensor(x[i:i + 1])).numpy()[0])
    out["x"] = x
    out["logprobs"] = np.stack(lps)
    out["softmax"] = torch.softmax(torch.tensor(out["logprobs"]), dim=1).numpy()
    out["mask1"] = np.concatenate(masks["drop1"])
    out["mask2"] = np.concatenate(masks["drop2"])
    for k, v in state.items():
        out["state_" + k] = v
    pool = sorted(glob.glob(os.path.join(REF, "resources/DABA/trigger_pool/*.wav")))[:4]
    for j, p in enumerate(pool):
        with wave.open(p) as w:
            assert w.getsampwidth() == 2 and w.getnchannels() == 1 and w.getframerate() == 16000
            out[f"pool{j}"] = np.frombuffer(w.readframes(w.getnframes()), dtype=np.int16).copy()
        out[f"pool{j}_name"] = np.array(os.path.basename(p))
    np.savez_compressed(os.path.join(HERE, "daba_golden.npz"), **out)
    print("wrote", sorted(out))


if __name__ == "__main__":
    main()
