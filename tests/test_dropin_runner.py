"""CPU: the drop-in boundary resolves the attack scripts' imports.

A stand-in tree shaped like the reference checkout (no reference files: every module is a stub
that only defines the imported names) holds a fake attack script whose import lines are exactly
those of badnets.py:10-15, ultrasonic.py:10-15, jingleback.py:10-15, daba.py:11-16 and
flowmur.py:11-16.  ``python -m abd_amd.run attack.py`` must resolve the accelerated names to
abd_amd and the rest (utils.visual_tools, the out-of-scope backbones) to the stand-in reference.
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

STUBS = {
    "prepare_dataset.py": ["MFCC", "load_clean_data", "BDDataset", "prepare_clean_dataset"],
    "utils/training_tools.py": ["train", "test", "EarlyStoppingModel", "clean_train", "clean_test"],
    "utils/models.py": ["smallcnn", "largecnn", "smalllstm", "lstmwithattention", "RNN", "ResNet", "ResidualBlock"],
    "utils/visual_tools.py": ["plot_loss", "plot_metrics"],
    "utils/random_tools.py": ["fix_random"],
    "utils/badnet_trigger.py": ["add_trigger_to_mfcc", "generate_trigger"],
    "utils/ultra_trigger.py": ["GenerateTrigger"],
    "utils/styles_trigger.py": ["get_boards", "poison_style"],
    "utils/daba_injection_tools.py": ["librosa_MFCC", "daba_poison_data"],
    "utils/daba_selection_tools.py": ["single_trigger_injection_db", "trigger_selection_hosts_selection"],
    "utils/flowmur_generate_trigger.py": ["pretrain_model", "generate_trigger"],
}

SCRIPT = '''
import json, sys
from prepare_dataset import MFCC, load_clean_data, BDDataset
from utils.random_tools import fix_random
from utils.badnet_trigger import add_trigger_to_mfcc, generate_trigger
from utils.training_tools import train, test, EarlyStoppingModel
from utils.visual_tools import plot_loss, plot_metrics
from utils.models import smallcnn, largecnn, smalllstm, lstmwithattention, RNN, ResNet, ResidualBlock
from utils.ultra_trigger import GenerateTrigger
from utils.styles_trigger import get_boards, poison_style
from utils.daba_injection_tools import librosa_MFCC, daba_poison_data
from utils.flowmur_generate_trigger import pretrain_model, generate_trigger as fm_generate_trigger
names = dict(MFCC=MFCC, load_clean_data=load_clean_data, BDDataset=BDDataset, fix_random=fix_random,
             add_trigger_to_mfcc=add_trigger_to_mfcc, generate_trigger=generate_trigger, train=train, test=test,
             EarlyStoppingModel=EarlyStoppingModel, plot_loss=plot_loss, plot_metrics=plot_metrics,
             smallcnn=smallcnn, largecnn=largecnn, ResNet=ResNet, GenerateTrigger=GenerateTrigger,
             get_boards=get_boards, poison_style=poison_style, librosa_MFCC=librosa_MFCC,
             daba_poison_data=daba_poison_data, pretrain_model=pretrain_model,
             fm_generate_trigger=fm_generate_trigger)
out = {k: [v.__module__, getattr(v, "__qualname__", "")] for k, v in names.items()}
out["__argv__"] = sys.argv[1:]
out["__name__"] = __name__
json.dump(out, open(sys.argv[1], "w"))
'''


def make_tree(tmp):
    for rel, names in STUBS.items():
        p = tmp / rel
        p.parent.mkdir(parents=True, exist_ok=True)
        body = "".join(f"class {n}:\n    ORIGIN = 'stand-in reference'\n" if n[0].isupper() else
                       f"def {n}(*a, **k):\n    return 'stand-in reference'\n" for n in names)
        p.write_text(body)
    (tmp / "attack.py").write_text(SCRIPT)


def test_runner_resolves_dropin_and_fallthrough(tmp_path):
    make_tree(tmp_path)
    out = tmp_path / "resolved.json"
    env = dict(os.environ, PYTHONPATH=ROOT, PYTHONDONTWRITEBYTECODE="1")
    r = subprocess.run([sys.executable, "-m", "abd_amd.run", "attack.py", str(out), "--flag"], cwd=tmp_path, env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    got = json.loads(out.read_text())
    mod = {k: v[0] for k, v in got.items() if not k.startswith("__")}
    assert got["__name__"] == "__main__" and got["__argv__"] == [str(out), "--flag"]
    expect = {
        "MFCC": "abd_amd.features", "BDDataset": "prepare_dataset", "load_clean_data": "prepare_dataset",
        "train": "abd_amd.training", "test": "abd_amd.training", "EarlyStoppingModel": "abd_amd.training",
        "smallcnn": "abd_amd.models", "add_trigger_to_mfcc": "abd_amd.triggers",
        "generate_trigger": "abd_amd.triggers", "GenerateTrigger": "abd_amd.triggers",
        "get_boards": "abd_amd.triggers", "poison_style": "abd_amd.triggers", "librosa_MFCC": "abd_amd.features",
        "daba_poison_data": "abd_amd.daba", "pretrain_model": "abd_amd.flowmur",
        "fm_generate_trigger": "abd_amd.flowmur", "fix_random": "utils.random_tools",
        # fall-through to the (stand-in) reference
        "plot_loss": "utils.visual_tools", "plot_metrics": "utils.visual_tools",
        "largecnn": "utils._reference_models", "ResNet": "utils._reference_models",
    }
    for k, v in expect.items():
        assert mod[k] == v, (k, mod[k], v)
    # the drop-in prepare_dataset / random_tools are ours, not the stand-in's
    r2 = subprocess.run([sys.executable, "-c", (
        "import sys; from abd_amd.run import setup_path; setup_path('attack.py');"
        "import prepare_dataset, utils.random_tools, utils.visual_tools;"
        "print(prepare_dataset.__file__); print(utils.random_tools.__file__); print(utils.visual_tools.__file__)")],
        cwd=tmp_path, env=env, capture_output=True, text=True, timeout=240)
    assert r2.returncode == 0, r2.stderr[-3000:]
    pd_file, rt_file, vt_file = r2.stdout.split()
    assert "dropin" in pd_file and "dropin" in rt_file
    assert vt_file == str(tmp_path / "utils" / "visual_tools.py")


def test_models_dropin_loads_other_backbones_lazily(tmp_path):
    """`from utils.models import smallcnn` does not execute the reference's utils/models.py;
    the first access to an out-of-scope backbone does (PEP 562 module __getattr__)."""
    make_tree(tmp_path)
    env = dict(os.environ, PYTHONPATH=ROOT, PYTHONDONTWRITEBYTECODE="1")
    r = subprocess.run([sys.executable, "-c", (
        "import sys; from abd_amd.run import setup_path; setup_path('attack.py');"
        "from utils.models import smallcnn; print('utils._reference_models' in sys.modules);"
        "from utils.models import largecnn; print('utils._reference_models' in sys.modules, largecnn())")],
        cwd=tmp_path, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    assert r.stdout.split() == ["False", "True", "stand-in", "reference"]


def test_runner_config_yaml_sets_argparse_defaults(tmp_path):
    """`abd_amd.run --config config/x.yaml script.py`: YAML keys become the script's argparse
    defaults (typed: load_clean_data False stays False), command-line flags win, num_epoches ->
    num_epochs, unknown keys are reported and ignored."""
    (tmp_path / "attack.py").write_text(
        "import argparse, json, sys\n"
        "p = argparse.ArgumentParser()\n"
        "p.add_argument('--model', type=str, default='largecnn')\n"
        "p.add_argument('--load_clean_data', type=bool, default=True)\n"
        "p.add_argument('--n_fft', type=int, default=400)\n"
        "p.add_argument('--num_epochs', type=int, default=300)\n"
        "p.add_argument('--learning_rate', type=float, default=0.001)\n"
        "a = p.parse_args()\n"
        "json.dump(vars(a), open(sys.argv[0] + '.json', 'w'))\n")
    (tmp_path / "cfg.yaml").write_text("model: smallcnn\nload_clean_data: False\nn_fft: 1103\nnum_epoches: 7\n"
                                       "learning_rate: 0.0001\ntrigger_pos: mid\n")
    env = dict(os.environ, PYTHONPATH=ROOT, PYTHONDONTWRITEBYTECODE="1")
    r = subprocess.run([sys.executable, "-m", "abd_amd.run", "--config", "cfg.yaml", "attack.py", "--n_fft", "2048"],
                       cwd=tmp_path, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    got = json.loads((tmp_path / "attack.py.json").read_text())
    assert got == {"model": "smallcnn", "load_clean_data": False, "n_fft": 2048, "num_epochs": 7,
                   "learning_rate": 0.0001}, got
    assert "trigger_pos" in r.stderr
