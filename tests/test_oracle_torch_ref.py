"""CPU: the torch-fp32 restatement of the reference path (oracle/torch_ref.py) is pinned before use.

* SmallCNN restatement == the reference smallcnn's golden eval log-probs (utils/models.py:17-65,
  tests/golden/golden_ref.npz from make_golden.py);
* its MFCC == the float64 oracle (both restate torchaudio T.MFCC, prepare_dataset.py:35-47);
* the convergence fixture's host features regenerate bit-for-bit here (the GPU replay test
  re-derives them on the GPU box and checks the same digest).
"""
import random

import numpy as np
import pytest
import torch

from golden_inputs import CONV_CFGS, EVAL_CFGS, convergence_data, data_digest, eval_inputs, make_state
from oracle import mfcc as om, torch_ref


@pytest.mark.parametrize("name", list(EVAL_CFGS))
def test_torch_ref_smallcnn_matches_reference_golden(golden, name):
    H, W, K, lf = EVAL_CFGS[name]
    st = make_state(H, W, K, lf, seed=1000 + H * 7 + W + K, trained_bn=True)
    m = torch_ref.SmallCNN(K, lf)
    m.load_state_dict({k: torch.tensor(v) for k, v in st.items()})
    m.eval()
    with torch.no_grad():
        y = m(torch.tensor(eval_inputs(H, W))).numpy()
    np.testing.assert_allclose(y, golden[f"eval_{name}_logprobs"], rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("cfg", [(16000, 40, 400, 160), (44100, 40, 1103, 441), (16000, 13, 2048, 512)])
def test_torch_ref_mfcc_matches_float64_oracle(cfg):
    sr, C, n_fft, hop = cfg
    from abd_amd import synth
    w, _ = synth.make_clips_np(6, sr, sr, 10, seed=9)
    mine = torch_ref.mfcc(torch.from_numpy(w), sr, C, n_fft, hop).numpy()
    ref = om.mfcc_model_input(w.astype(np.float64), sr, C, n_fft, hop)
    err = np.abs(mine - ref).reshape(6, -1).max(1) / np.abs(ref).reshape(6, -1).max(1)
    assert err.max() < 1e-4, err


def test_convergence_features_regenerate(conv_golden):
    random.seed(35)
    d = convergence_data("badnets")
    assert np.array_equal(data_digest(d), conv_golden["badnets_data_digest"])
    c = CONV_CFGS["badnets"]
    assert d["bd_x"].shape == (c["n_train"], 1, 101, 40) and int(d["ind"].sum()) == int(c["n_train"] * 0.1)
    # badnets.py:66-77: target-class test clips stay clean with indicator 0, every label is the target
    assert np.all(d["bt_y"] == 2) and np.array_equal(d["bt_ind"], (d["clean_y"] != 2).astype(np.int64))
