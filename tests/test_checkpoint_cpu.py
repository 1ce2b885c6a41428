"""CPU: checkpoints written by the drop-in are the reference's format.

* the abd ``smallcnn`` state_dict loads strictly into the reference's ``utils.models.smallcnn``
  (imported from /root/reference when present: the build container) and both forwards agree;
* the whole-module pickle ``EarlyStoppingModel`` writes (utils/training_tools.py:44-50,
  consumed by fp.py:124-125 / ft_reg.py:237-238 / tsbd.py:255-256) round-trips on the host.
The GPU half (a trained model's checkpoint reloaded, identical eval log-probs) is
tests/test_gpu_dropin_loop.py.
"""
import os
import sys

import pytest
import torch

from abd_amd.models import smallcnn
from abd_amd.training import EarlyStoppingModel
from oracle import torch_ref

REF = os.environ.get("ABD_REFERENCE", "/root/reference")


def _model(K=10, lf=3072, seed=123):
    torch.manual_seed(seed)
    return smallcnn(K, lf)


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "utils")), reason="reference checkout not present")
@pytest.mark.parametrize("K,lf", [(10, 3072), (35, 3072), (10, 896), (10, 224)])
def test_state_dict_loads_into_reference_smallcnn(K, lf):
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    try:
        import utils.models as ref_models
    finally:
        sys.path.remove(REF)
    m = _model(K, lf)
    sd = m.state_dict()
    torch.manual_seed(123)
    ref = ref_models.smallcnn(K, lf)
    # same init under the same seed (the reference builds its model before fix_random)
    for k, v in ref.state_dict().items():
        assert torch.equal(v, sd[k]), k
    ref.load_state_dict(sd, strict=True)
    ref.eval()
    t = torch_ref.SmallCNN(K, lf)
    t.load_state_dict(sd, strict=True)
    t.eval()
    H, W = {3072: (101, 40), 896: (32, 40), 224: (32, 13)}[lf]
    x = torch.randn(3, 1, H, W) * 20
    with torch.no_grad():
        assert torch.allclose(ref(x), t(x), rtol=1e-5, atol=1e-5)


def test_whole_module_checkpoint_round_trip(tmp_path):
    m = _model()
    es = EarlyStoppingModel(patience=2, verbose=False, path=str(tmp_path / "checkpoint.pt"))
    es(1.0, m)      # first call always saves (training_tools.py:31-33)
    es(1.5, m)      # no improvement: counter 1
    es(2.0, m)      # counter 2 -> early stop
    assert es.early_stop and es.counter == 2
    loaded = torch.load(str(tmp_path / "checkpoint.pt"), weights_only=False)   # written by this test
    assert isinstance(loaded, smallcnn) and loaded._engine is None
    a, b = m.state_dict(), loaded.state_dict()
    assert sorted(a) == sorted(b) and all(torch.equal(a[k], b[k]) for k in a)
