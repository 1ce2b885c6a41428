"""CPU: the resident-loader fast path yields the loader's own batches (resident.py).

Same rows in the same order as ``for batch in loader`` and the same consumption of torch's global
RNG afterwards (the reference's dropout masks are drawn from it between batches,
utils/training_tools.py:59-70), for the datasets the scripts build (badnets.py:100-108)."""
import torch
from torch.utils.data import DataLoader, TensorDataset

from abd_amd import resident as R


class BDDataset(torch.utils.data.Dataset):
    """prepare_dataset.py:13-33's item contract (recognised by class name and module)."""

    def __init__(self, mfcc_list, label_list, poison_index):
        self.mfcc_list, self.label_list, self.poison_index = mfcc_list, label_list, poison_index

    def __len__(self):
        return len(self.mfcc_list)

    def __getitem__(self, index):
        return {"mfcc": self.mfcc_list[index], "label": self.label_list[index],
                "poison_indicator": self.poison_index[index]}


BDDataset.__module__ = "prepare_dataset"


class Custom(BDDataset):
    def __getitem__(self, index):
        return super().__getitem__(index)


def _data(n=203):
    g = torch.Generator().manual_seed(1)
    return (torch.randn(n, 1, 5, 3, generator=g), torch.randint(0, 10, (n,), generator=g),
            torch.randint(0, 2, (n,), generator=g))


def _compare(loader, dict_items):
    torch.manual_seed(123)
    ref = []
    for item in loader:
        ref.append((item["mfcc"], item["label"], item["poison_indicator"]) if dict_items else (item[0], item[1], None))
    after_ref = torch.rand(4)
    torch.manual_seed(123)
    ts = R._sources(loader.dataset, dict_items)
    assert ts is not None
    got = list(R._iterate(loader, R._Resident(ts, torch.device("cpu"))))
    after_got = torch.rand(4)
    assert torch.equal(after_ref, after_got), "different consumption of the global RNG"
    assert len(got) == len(ref)
    for (x, y, i), (rx, ry, ri) in zip(got, ref):
        assert torch.equal(x, rx.float()) and torch.equal(y, ry.long())
        assert (i is None and ri is None) or torch.equal(i, ri.long())


def test_bddataset_shuffled_batches_and_rng():
    x, y, i = _data()
    _compare(DataLoader(BDDataset(x, y, i), batch_size=32, shuffle=True), True)
    _compare(DataLoader(BDDataset(x, y, i), batch_size=64, shuffle=False), True)


def test_tensordataset_batches_and_rng():
    x, y, _ = _data()
    _compare(DataLoader(TensorDataset(x.double(), y), batch_size=50, shuffle=True), False)


def test_unsupported_loaders_fall_back():
    x, y, i = _data()
    cpu = torch.device("cpu")
    cuda = torch.device("cuda", 0)
    assert R.resident_batches(DataLoader(BDDataset(x, y, i), batch_size=8), cpu, True) is None   # host device
    assert R._sources(Custom(x, y, i), True) is None                        # overridden item contract
    assert R._sources(TensorDataset(x, y), True) is None                    # tuple items where dicts are expected
    assert R._sources(BDDataset(x, y, i), False) is None
    assert R._sources(BDDataset(x.numpy(), y, i), True) is None             # numpy-backed
    for kw in (dict(num_workers=1), dict(collate_fn=lambda b: b)):
        assert R.resident_batches(DataLoader(BDDataset(x, y, i), batch_size=8, **kw), cuda, True) is None


def test_cache_key_tracks_in_place_writes():
    x, y, i = _data()
    k0 = R._key((x, y, i))
    x[0, 0, 0, 0] += 1.0      # e.g. add_trigger_to_mfcc's in-place patch (badnet_trigger.py:25)
    assert R._key((x, y, i)) != k0


def test_fast_path_falls_back_without_next_index(monkeypatch):
    """a torch whose DataLoader iterator lacks _next_index() gets the host loader, not an
    AttributeError inside train()."""
    from torch.utils.data.dataloader import _BaseDataLoaderIter
    from abd_amd import resident
    ds = torch.utils.data.TensorDataset(torch.zeros(4, 1, 2, 2), torch.zeros(4, dtype=torch.long))
    loader = torch.utils.data.DataLoader(ds, batch_size=2)
    monkeypatch.delattr(_BaseDataLoaderIter, "_next_index")
    assert resident.resident_batches(loader, torch.device("cuda", 0), False) is None
