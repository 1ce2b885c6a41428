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


def _write_checkpoint(tmp_path, K=10, lf=3072):
    m = _model(K, lf)
    m.eval()
    es = EarlyStoppingModel(patience=2, verbose=False, path=str(tmp_path / "checkpoint.pt"))
    es(1.0, m)      # first call always saves (training_tools.py:31-33)
    es(1.5, m)      # no improvement: counter 1
    es(2.0, m)      # counter 2 -> early stop
    assert es.early_stop and es.counter == 2
    return m, str(tmp_path / "checkpoint.pt")


def test_whole_module_checkpoint_round_trip(tmp_path):
    """Under the drop-in (abd_amd.run puts dropin/ first: flowmur.py:55 reloads its benign model),
    the pickle resolves utils.models.smallcnn to the accelerated class."""
    m, path = _write_checkpoint(tmp_path)
    from conftest import load_dropin_checkpoint
    loaded = load_dropin_checkpoint(path)
    assert isinstance(loaded, smallcnn) and loaded._engine is None and loaded._step == 0
    assert loaded.gemm_precision == "f32split" and not loaded.training
    a, b = m.state_dict(), loaded.state_dict()
    assert sorted(a) == sorted(b) and all(torch.equal(a[k], b[k]) for k in a)


_CONSUMER = r"""
import sys, json
sys.dont_write_bytecode = True
sys.path[:] = [p for p in sys.path if p and 'repo' not in p]
sys.path.insert(0, {ref!r})
import torch, torch.nn as nn
from torch.nn.utils import prune
m = torch.load({path!r}, map_location='cpu', weights_only=False)   # fp.py:125 (our own file)
out = {{"module": type(m).__module__, "cls": type(m).__name__,
        "abd_loaded": any(k.startswith('abd_amd') for k in sys.modules)}}
m.eval()
m.requires_grad_(False)
import copy
mc = copy.deepcopy(m)                                              # fp.py:128
name, last = list(mc.named_children())[-1]                         # fp.py:137
out["last_child"] = name
fired = []
h = mc.fc2.register_forward_hook(lambda mod, i, o: fired.append(tuple(i[0].shape)))
x = torch.load({xpath!r}, weights_only=True)
with torch.no_grad():
    y = mc(x)
out["hook"] = fired
h.remove()
mask = torch.ones_like(mc.fc1.weight)
mask[:, :7] = 0
prune.custom_from_mask(mc.fc1, name="weight", mask=mask)          # fp.py:171
with torch.no_grad():
    yp = mc(x)
out["pruned_has_orig"] = hasattr(mc.fc1, "weight_orig")
torch.save({{"y": y, "yp": yp}}, {ypath!r})
print(json.dumps(out))
"""


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "utils")), reason="reference checkout not present")
@pytest.mark.parametrize("K,lf,H,W", [(10, 3072, 101, 40), (35, 3072, 100, 40), (10, 896, 32, 40)])
def test_checkpoint_loads_as_reference_class_without_abd(tmp_path, K, lf, H, W):
    """the defenses (fp.py, ft_reg.py, tsbd.py, correlation_analysis.py) torch.load the
    checkpoint with only the reference on sys.path and operate on its submodules."""
    import json
    import subprocess
    m, path = _write_checkpoint(tmp_path, K, lf)
    torch.manual_seed(3)
    x = torch.randn(4, 1, H, W) * 20
    xpath, ypath = str(tmp_path / "x.pt"), str(tmp_path / "y.pt")
    torch.save(x, xpath)
    code = _CONSUMER.format(ref=REF, path=path, xpath=xpath, ypath=ypath)
    env = {k: v for k, v in os.environ.items() if k != "PYTHONPATH"}
    env["PYTHONDONTWRITEBYTECODE"] = "1"
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, cwd=str(tmp_path),
                       timeout=300)
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["module"] == "utils.models" and out["cls"] == "smallcnn" and not out["abd_loaded"], out
    assert out["last_child"] == "softmax"                 # the reference's own child order
    assert out["hook"] == [[4, 128]] and out["pruned_has_orig"], out
    ys = torch.load(ypath, weights_only=True)
    t = torch_ref.SmallCNN(K, lf)
    t.load_state_dict(m.state_dict(), strict=True)
    t.eval()
    with torch.no_grad():
        exp = t(x)
        t.fc1.weight[:, :7] = 0
        exp_p = t(x)
    assert torch.allclose(ys["y"], exp, rtol=1e-5, atol=1e-5)
    assert torch.allclose(ys["yp"], exp_p, rtol=1e-5, atol=1e-5)


def _pickle_ops(path):
    import pickletools
    import zipfile
    z = zipfile.ZipFile(path)
    data = z.read([n for n in z.namelist() if n.endswith("data.pkl")][0])
    return [(op.name, arg) for op, arg, _ in pickletools.genops(data)
            if op.name in ("GLOBAL", "STACK_GLOBAL", "NEWOBJ", "REDUCE", "BUILD")]


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "utils")), reason="reference checkout not present")
def test_checkpoint_opcodes_equal_reference_torch_save(tmp_path):
    """the stream is the reference's own torch.save(model) (utils/training_tools.py:49) --
    GLOBAL utils.models smallcnn + NEWOBJ, no import_module / getattr REDUCE calls -- opcode for opcode."""
    m, path = _write_checkpoint(tmp_path, 10, 896)
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    try:
        import utils.models as ref_models
    finally:
        sys.path.remove(REF)
    ref = ref_models.smallcnn(10, 896)
    ref.load_state_dict(m.state_dict())
    ref.eval()
    rpath = str(tmp_path / "ref.pt")
    torch.save(ref, rpath)
    ours, theirs = _pickle_ops(path), _pickle_ops(rpath)
    assert ours[0] == ("GLOBAL", "utils.models smallcnn") and ours[1][0] == "NEWOBJ"
    assert not any(a in ("importlib import_module", "builtins getattr") for _, a in ours)
    assert ours == theirs


_SAFE_CONSUMER = r"""
import sys, json, collections
sys.dont_write_bytecode = True
sys.path[:] = [p for p in sys.path if p and 'repo' not in p]
sys.path.insert(0, {ref!r})
import torch, torch.nn as nn
import utils.models as rm
allow = [rm.smallcnn, nn.Conv2d, nn.BatchNorm2d, nn.MaxPool2d, nn.Dropout, nn.Flatten, nn.Linear, nn.Softmax,
         collections.OrderedDict, set]
with torch.serialization.safe_globals(allow):
    m = torch.load({path!r}, map_location='cpu')            # weights_only=True: torch>=2.6 default
m.eval()
x = torch.load({xpath!r}, weights_only=True)
with torch.no_grad():
    torch.save(m(x), {ypath!r})
print(json.dumps({{"cls": type(m).__module__ + "." + type(m).__name__,
                   "abd_loaded": any(k.startswith('abd_amd') for k in sys.modules)}}))
"""


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "utils")), reason="reference checkout not present")
def test_checkpoint_loads_weights_only_with_reference_allowlist(tmp_path):
    """torch.load's weights_only=True default accepts the checkpoint once the consumer
    allowlists the reference's classes -- exactly what it needs for the reference's own pickle."""
    import json
    import subprocess
    m, path = _write_checkpoint(tmp_path, 10, 896)
    torch.manual_seed(4)
    x = torch.randn(3, 1, 32, 40) * 20
    xpath, ypath = str(tmp_path / "x.pt"), str(tmp_path / "y.pt")
    torch.save(x, xpath)
    code = _SAFE_CONSUMER.format(ref=REF, path=path, xpath=xpath, ypath=ypath)
    env = {k: v for k, v in os.environ.items() if k != "PYTHONPATH"}
    env["PYTHONDONTWRITEBYTECODE"] = "1"
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, cwd=str(tmp_path),
                       timeout=300)
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out == {"cls": "utils.models.smallcnn", "abd_loaded": False}, out
    t = torch_ref.SmallCNN(10, 896)
    t.load_state_dict(m.state_dict(), strict=True)
    t.eval()
    with torch.no_grad():
        assert torch.allclose(torch.load(ypath, weights_only=True), t(x), rtol=1e-5, atol=1e-5)
