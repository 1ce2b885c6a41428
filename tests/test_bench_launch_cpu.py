"""CPU: bench.py's launch plumbing (`--gpus N` without a launcher spawns the N ranks itself; under a
launcher WORLD_SIZE must equal N).  No GPU: the parent process never imports torch, and the spawned
command here is a stand-in that reports its rendezvous environment."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_resolve_world():
    assert bench.resolve_world(1, {}) == (1, False)
    assert bench.resolve_world(4, {}) == (4, True)
    assert bench.resolve_world(2, {"WORLD_SIZE": "2"}) == (2, False)
    with pytest.raises(SystemExit):
        bench.resolve_world(2, {"WORLD_SIZE": "1"})
    with pytest.raises(SystemExit):
        bench.resolve_world(1, {"WORLD_SIZE": "8"})
    with pytest.raises(SystemExit):
        bench.resolve_world(0, {})


def test_rank_envs():
    envs = bench.rank_envs(3, 29999, base={"X": "1"})
    assert [e["RANK"] for e in envs] == ["0", "1", "2"]
    assert [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2"]
    for e in envs:
        assert e["WORLD_SIZE"] == "3" and e["MASTER_ADDR"] == "127.0.0.1" and e["MASTER_PORT"] == "29999"
        assert e["X"] == "1"


def test_spawn_ranks_runs_n_children(tmp_path):
    out = tmp_path / "r"
    code = ("import os, json; open(%r + os.environ['RANK'], 'w').write(json.dumps({k: os.environ[k] for k in "
            "('RANK', 'LOCAL_RANK', 'WORLD_SIZE', 'MASTER_ADDR', 'MASTER_PORT')}))" % str(out))
    assert bench.spawn_ranks(2, [sys.executable, "-c", code], poll_s=0.01) == 0
    got = [json.load(open(str(out) + str(r))) for r in range(2)]
    assert [g["RANK"] for g in got] == ["0", "1"] and all(g["WORLD_SIZE"] == "2" for g in got)
    assert got[0]["MASTER_PORT"] == got[1]["MASTER_PORT"]


def test_spawn_ranks_failing_rank_stops_the_others():
    # rank 1 fails at once; rank 0 would otherwise wait 60 s (a rank stuck in a collective)
    code = "import os, sys, time; r = int(os.environ['RANK']); sys.exit(3) if r == 1 else time.sleep(60)"
    import time
    t0 = time.time()
    assert bench.spawn_ranks(2, [sys.executable, "-c", code], poll_s=0.01) == 3
    assert time.time() - t0 < 30


def test_bench_rejects_world_size_mismatch():
    env = dict(os.environ, WORLD_SIZE="1")
    res = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=env, cwd=ROOT,
                         capture_output=True, text=True, timeout=60)
    assert res.returncode != 0
    assert "disagrees with --gpus 2" in res.stderr


def test_spawn_ranks_relays_only_rank0_json(capfd):
    """Collective libraries print banners to stdout (gloo: "[Gloo] Rank 0 is connected to ..."): only
    rank 0's JSON line reaches stdout, the rest goes to stderr."""
    code = ("import os, sys; r = os.environ['RANK']; print('[Gloo] Rank ' + r + ' is connected'); "
            "print('{\"rank\": ' + r + '}') if r == '0' else print('{\"rank\": 9}'); sys.stdout.flush()")
    assert bench.spawn_ranks(2, [sys.executable, "-c", code], poll_s=0.01) == 0
    out, err = capfd.readouterr()
    assert out.strip().splitlines() == ['{"rank": 0}'], out
    assert "[Gloo] Rank 0" in err and "[Gloo] Rank 1" in err and '{"rank": 9}' in err
