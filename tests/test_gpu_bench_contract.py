"""bench.py's output contract, as the round-end driver reads it (task brief, "Maintain bench.py"):
one JSON line on rank 0 with the metric / config of BASELINE.json, the whole-job value, and the
`roofline` and `cpu_baseline` objects.  Runs a short bench in a child process (the same command
shape the driver uses at N = 1) and checks the line's fields and their arithmetic."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_json_line_contract():
    with open(os.path.join(ROOT, "BASELINE.json")) as f:
        base = json.load(f)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "8", "--warmup", "2", "--profile-steps", "1",
           "--dropin-batches", "2", "--cpu-train", "512"]
    res = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert res.returncode == 0, res.stderr[-2000:]
    lines = [ln for ln in res.stdout.strip().splitlines() if ln.startswith("{")]
    assert len(lines) == 1, res.stdout[-2000:]
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["metric"] == base["metric"]
    assert d["n_gpus"] == 1 and d["steps"] == 8 and d["warmup"] == 2 and d["scaling"] == "weak"
    assert d["higher_is_better"] is True and d["vs_baseline"] is None and d["data"] == "synthetic"
    B = d["config"]["per_gpu_batch"]
    assert B == 512 and "workload" in d["config"]
    # value = utterances per second of the whole job = B * N / ms_per_step (4 significant digits rounded)
    assert abs(d["value"] - B * 1e3 / d["ms_per_step"]) <= 1e-3 * d["value"]
    r = d["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in r, k
    assert r["bound"] in ("hbm", "mfma") and r["unit"] in ("GB/s", "TFLOP/s")
    assert 0.0 < r["frac"] < 1.0 and abs(r["frac"] - r["achieved"] / r["peak"]) <= 1e-3
    # the dominant kernel's average launch lies inside the step
    assert 0.0 < r["avg_launch_ms"] < d["ms_per_step"]
    c = d["cpu_baseline"]
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in c, k
    assert c["kind"] in ("port", "reference") and c["value"] > 0 and c["cores"] >= 1


def test_bench_gpus2_spawns_two_ranks():
    """`bench.py --gpus 2` with no launcher: the parent spawns two ranks itself (here both
    on the one GPU, gloo), rank 0 prints ONE line with n_gpus 2 / dp2 and the whole-job value."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-backend", "gloo", "--steps", "8",
           "--warmup", "2", "--profile-steps", "1", "--no-cpu", "--dropin-batches", "0", "--n-train", "2048"]
    res = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert res.returncode == 0, res.stderr[-2000:]
    lines = [ln for ln in res.stdout.strip().splitlines() if ln.startswith("{")]
    assert len(lines) == 1, res.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "dp2" and d["config"]["global_batch"] == 1024
    assert abs(d["value"] - 1024 * 1e3 / d["ms_per_step"]) <= 1e-3 * d["value"]
    assert abs(d["value_per_gpu"] - d["value"] / 2) <= 0.1 + 1e-3 * d["value"]
