"""CPU: the resident pipeline's index work is the reference's, bit for bit.

* poison rows: ``random.sample`` after ``fix_random()`` (badnets.py:50-51, ultrasonic.py:70-71,
  jingleback.py:66-67); FlowMur's ``np.random.choice`` + per-clip ``random.randint``
  (flowmur.py:58-81);
* epoch order: ``DataLoader(shuffle=True)`` with ``test()`` iterating two shuffled loaders
  between training epochs (badnets.py:105-108, :146-148) -- compared with real DataLoaders.
"""
import random

import numpy as np
import torch

from abd_amd.pipeline import LoaderOrder, attack_config, poison_schedule


def test_badnets_poison_rows_are_random_sample_after_fix_random():
    for N in (100, 2048, 20480):
        random.seed(35)  # fix_random(), utils/random_tools.py:5-18
        ref = random.sample(list(range(N)), int(N * 0.1))
        for name in ("badnets", "ultrasonic", "jingleback"):
            rows, pos, _ = poison_schedule(attack_config(name), np.zeros(N, np.int64), seed=35)
            assert pos is None
            assert rows.tolist() == ref


def test_flowmur_poison_rows_and_positions():
    cfg = attack_config("flowmur")
    r = np.random.Generator(np.random.PCG64(4))
    for N in (400, 8000):
        labels = r.integers(0, 10, N).astype(np.int64)
        random.seed(35)
        np.random.seed(35)
        n_tr = N - int(np.ceil(0.2 * N))
        if n_tr >= 5000:
            random.sample(range(n_tr), 5000)                       # flowmur.py:60
        tgt = np.where(labels == 2)[0]
        ref_rows = np.random.choice(tgt, int(tgt.shape[0] * 0.1), replace=False)   # :74-76
        ref_pos = [random.randint(0, 16000 - 8000) for _ in ref_rows]              # :81
        rows, pos, pr = poison_schedule(cfg, labels, seed=35, trigger_len=8000)
        assert rows.tolist() == ref_rows.tolist() and pos.tolist() == ref_pos
        # the test-set window draws continue the same python stream (flowmur.py:102)
        assert pr.randint(0, 8000) == random.randint(0, 8000)


class _Set(torch.utils.data.Dataset):
    def __init__(self, n):
        self.n = n

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        return i


def test_epoch_order_matches_shuffled_dataloaders():
    """Three epochs of eval_model's loop: train loader, then test() over two shuffled loaders."""
    N, B = 1000, 256
    torch.manual_seed(35)
    train = torch.utils.data.DataLoader(_Set(N), batch_size=B, shuffle=True)
    clean = torch.utils.data.DataLoader(_Set(200), batch_size=B, shuffle=True)
    bd = torch.utils.data.DataLoader(_Set(200), batch_size=B, shuffle=True)
    ref = []
    for _ in range(3):
        ref.append(torch.cat(list(train)).tolist())
        for _ in clean:
            pass
        for _ in bd:
            pass
    lo = LoaderOrder(N, seed=35)
    mine = [lo.next_epoch().tolist() for _ in range(3)]
    assert mine == ref
