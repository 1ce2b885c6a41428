"""CPU: the C-ABI library loads and exports every header symbol; host-side logic of the package."""
import os
import re
import tempfile

import numpy as np
import pytest
import torch

import abd_amd
from abd_amd import _lib as L

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    txt = open(os.path.join(ROOT, "include", "abd.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(abd_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    lib = abd_amd.load_library()
    names = header_functions()
    assert len(names) >= 25
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    assert set(L.EXPORTS) <= set(names)
    assert lib.abd_version() >= 1


def test_library_rejects_bad_arguments_without_gpu():
    import ctypes as C
    lib = abd_amd.load_library()
    h = C.c_void_p()
    assert lib.abd_smallcnn_create(101, 40, 100, 0, C.byref(h)) == 1002      # >64 classes unsupported
    assert b"num_classes" in lib.abd_last_error()
    assert lib.abd_smallcnn_create(101, 40, 10, 0, C.byref(h)) == 0
    assert lib.abd_smallcnn_param_count(h) == 419946
    assert lib.abd_smallcnn_flat_features(h) == 3072
    off = (C.c_int64 * 17)()
    lib.abd_smallcnn_param_offsets(h, off)
    assert list(off)[:3] == [0, 256, 320] and off[16] == 419946
    assert lib.abd_smallcnn_workspace_offset(h, 8, b"nonexistent") == -1
    assert lib.abd_smallcnn_workspace_offset(h, 8, b"p1") == 0
    lib.abd_smallcnn_destroy(h)
    for (H, W, lf) in ((32, 40, 896), (32, 13, 224), (100, 40, 3072)):
        assert lib.abd_smallcnn_create(H, W, 10, 0, C.byref(h)) == 0
        assert lib.abd_smallcnn_flat_features(h) == lf                       # attack_config.txt:11-23
        lib.abd_smallcnn_destroy(h)
    # sampled profiler brackets (bench.py --profile-every): the period is checked before any HIP call
    assert lib.abd_profile_start_every(1, 16, 0) == 1001 and lib.abd_profile_start_every(1, -1, 4) == 1001


def test_smallcnn_init_and_state_dict_match_reference(golden):
    from abd_amd.models import smallcnn
    from test_oracle_golden import _digest
    for K, lf in ((10, 3072), (35, 3072), (10, 224)):
        torch.manual_seed(123)
        m = smallcnn(K, lf)
        sd = m.state_dict()
        keys = sorted(k[len(f"init_{K}_{lf}_"):] for k in golden if k.startswith(f"init_{K}_{lf}_"))
        assert sorted(sd) == keys
        for k in keys:
            np.testing.assert_array_equal(_digest(sd[k].numpy(), 15), golden[f"init_{K}_{lf}_{k}"])


def test_cpu_forward_fails_loudly():
    from abd_amd.models import smallcnn
    with pytest.raises(L.AbdError):
        smallcnn(10, 3072)(torch.zeros(2, 1, 101, 40))


def test_badnets_trigger_api(golden):
    from abd_amd import triggers
    t = triggers.generate_trigger(40, 101, 5, save=False)
    np.testing.assert_array_equal(t, golden["badnet_trigger_101x40"])
    np.testing.assert_array_equal(triggers.generate_trigger(13, 32, 3, 1, 2, save=False),
                                  golden["badnet_trigger_32x13_s3_d1"])
    assert triggers.patch_spec(t) == (96, 101, 35, 40, -200.0)
    from abd_amd.pipeline import attack_config
    assert attack_config("badnets").patch == (96, 101, 35, 40, -200.0)
    m = np.zeros((1, 101, 40), np.float32)
    assert triggers.add_trigger_to_mfcc(m, t) is m and (m[0, 96:, 35:] == -200).all() and m.sum() == -200 * 25


def test_ultrasonic_trigger_api_known_answer(wavs):
    from abd_amd import triggers
    g = triggers.GenerateTrigger(60, "end", cont=True).trigger()
    np.testing.assert_array_equal(g[0], wavs["ante_int16"].astype(np.float32) / 32768.0)   # utils/ante.wav
    with pytest.raises(triggers.TriggerInfeasible):
        triggers.GenerateTrigger(0, "mid")
    with pytest.raises(triggers.TriggerInfeasible):
        triggers.GenerateTrigger(30, "middle")
    from oracle import triggers as otr
    base = wavs["ultrasonic_trigger_int16"].astype(np.float64)[None] / 32768.0
    for size in (15, 30, 45, 60):
        for pos in ("start", "mid", "end"):
            for cont in (True, False):
                np.testing.assert_array_equal(triggers.GenerateTrigger(size, pos, cont).trigger()[0],
                                              otr.ultrasonic_gate(base, size, pos, cont)[0].astype(np.float32))


def test_pydub_dbfs_matches_oracle():
    from abd_amd import triggers
    from oracle import triggers as otr
    x = np.random.default_rng(0).integers(-20000, 20000, 16000).astype(np.int16)
    assert triggers.dbfs_int16(x) == pytest.approx(otr.pydub_dbfs(x))
    assert triggers.dbfs_int16(np.zeros(10, np.int16)) == -np.inf


def test_wav_io_and_label_sets():
    from abd_amd import io
    x = np.random.default_rng(1).integers(-32768, 32767, 1000).astype(np.int16)
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "a.wav")
        io.write_wav_int16(p, x, 16000)
        y, sr = io.read_wav_int16(p)
        f, _ = io.read_wav(p)
    assert sr == 16000 and np.array_equal(x, y) and np.allclose(f, x / 32768.0)
    assert [len(io.LABEL_SETS[k][1]) for k in ("SCDv1-10", "SCDv1-30", "SCDv2-10", "SCDv2-26", "SCDv2-35")] == \
        [10, 30, 10, 26, 35]
    tr, te = io.train_test_split_35(100)
    assert len(te) == 20 and len(set(tr) | set(te)) == 100


def test_fused_path_selection():
    from abd_amd.models import smallcnn
    from abd_amd.training import fusable
    m = smallcnn(10, 3072)
    ce = torch.nn.CrossEntropyLoss()
    assert fusable(m, torch.optim.Adam(m.parameters(), lr=1e-4), ce)
    assert not fusable(m, torch.optim.SGD(m.parameters(), lr=1e-4), ce)
    assert not fusable(m, torch.optim.Adam(m.parameters(), lr=1e-4, weight_decay=1e-2), ce)
    assert not fusable(m, torch.optim.Adam(m.parameters(), lr=1e-4), torch.nn.CrossEntropyLoss(label_smoothing=0.1))
    assert not fusable(m, torch.optim.Adam(list(m.parameters())[:3], lr=1e-4), ce)


def test_early_stopping_semantics():
    from abd_amd.training import EarlyStoppingModel
    saved = []
    es = EarlyStoppingModel(patience=2, path=os.devnull, trace_func=lambda *a: None)
    es.save_checkpoint = lambda loss, model: saved.append(loss)
    for v in (1.0, 0.9, 0.95, 0.92, 0.91):
        es(v, None)
    assert saved == [1.0, 0.9] and es.early_stop


def test_dropin_modules_import():
    import subprocess
    import sys
    code = ("import sys; sys.path.insert(0, 'audio-backdoor-attack_amd/dropin');"
            "import prepare_dataset, utils.models, utils.training_tools, utils.badnet_trigger, utils.ultra_trigger,"
            "utils.random_tools, utils.daba_selection_tools, utils.flowmur_generate_trigger, utils.styles_trigger;"
            "from prepare_dataset import MFCC, BDDataset, load_clean_data;"
            "from utils.training_tools import train, test, EarlyStoppingModel;"
            "from utils.models import smallcnn; print('ok')")
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True)
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr
