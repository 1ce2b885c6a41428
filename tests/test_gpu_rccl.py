"""GPU: the data-parallel step's collectives through RCCL (torch.distributed "nccl") on one GPU.

The DP tests in test_gpu_dp.py run two ranks over gloo (RCCL needs one GPU per rank and the test
box has one).  gloo never exercises ProcessGroupNCCL's stream semantics, so here a world-size-1
RCCL group drives every collective of ResidentTrainer's data-parallel step (collectives=True):

* OverlappedGradAllReduce: libabd records the fc-gradient hipEvent mid-backward, a side stream
  waits on it and issues the fc-tail all-reduce there (async Work), the conv-head all-reduce
  follows on the compute stream, ``Work.wait()`` joins both stream-side, then the separate Adam;
* SyncBatchNorm: libabd's six ctypes callbacks per step issue ``dist.all_reduce`` on the current
  stream between two of its launches;
* reduce_metrics / broadcast_state (the initial parameter, buffer and dropout-seed broadcast).

Parameters, BN buffers and the epoch metrics must equal (1e-6) the plain one-process step's for the
collectives-only step (the same kernels, Adam after the all-reduce), and the same SyncBN step run
over a one-rank gloo group for the SyncBN step (SyncBN has its own launches: no BN1 fold, the
activation passes, the unfused fc head).
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(port, attack, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        import sys
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        sys.path.insert(0, root)
        import torch.distributed as dist
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
        import abd_amd
        from abd_amd import synth
        from abd_amd.models import smallcnn
        from abd_amd.pipeline import ResidentTrainer, attack_config
        abd_amd.load_library()
        cfg = attack_config(attack)
        B, K, steps = 96, 10, 4
        waves, labels = synth.make_clips_torch(3 * B + 17, cfg.sample_rate, cfg.length, K, seed=41, device=dev)
        trigger = None
        if cfg.clean_label:   # FlowMur: target-class clips to poison and a trigger (flowmur.py:67-85)
            import numpy as np
            labels[: labels.numel() // 4] = cfg.target_label
            trigger = (0.05 * np.random.default_rng(1).standard_normal(8000)).astype(np.float32)

        gloo = dist.new_group([0], backend="gloo")

        def run(dp, sync_bn, pg=None):
            torch.manual_seed(35)
            model = smallcnn(K, cfg.linear_features).to(dev)
            opt = torch.optim.Adam(model.parameters(), lr=1e-3)
            tr = ResidentTrainer(cfg, waves, labels, model, opt, B, trigger=trigger, seed=35, collectives=dp,
                                 sync_bn=sync_bn, process_group=pg)
            for _ in range(steps):   # crosses the epoch's 17-row tail
                tr.step()
            m = tr.read_metrics()
            tr.sync_buffers()
            torch.cuda.synchronize()
            eng = model._engine
            return eng.params.clone(), eng.running.clone(), eng.nbt.clone(), m, tr

        # collectives only: against the plain single-rank step (the same kernels)
        # SyncBN: against the same SyncBN step over a one-rank gloo group (the SyncBN path has its own
        # kernels -- no BN1 fold, activation passes -- so the reference is that path, not the fused one)
        plain = run(False, False)
        gloo_sync = run(True, True, gloo)
        res = {"backend": dist.get_backend()}
        for sync_bn in (False, True):
            p0, r0, n0, m0, _ = gloo_sync if sync_bn else plain
            p1, r1, n1, m1, tr = run(True, sync_bn)
            nrel = lambda a, b: float((a - b).norm() / b.norm())  # noqa: E731
            res[sync_bn] = {"params": nrel(p1, p0), "running": nrel(r1, r0), "nbt": torch.equal(n1, n0),
                            "loss": abs(m1["loss"] - m0["loss"]) / m0["loss"], "acc": (m1["acc"], m0["acc"]),
                            "samples": (m1["samples"], m0["samples"]),
                            "bn_calls": tr.bn_sync.calls if tr.bn_sync is not None else None,
                            "reducer": tr.reducer is not None}
        q.put((res, None))
        dist.destroy_process_group()
    except Exception:
        import traceback
        q.put((None, traceback.format_exc()))
        raise


@pytest.mark.parametrize("attack", ["badnets", "flowmur"])
def test_rccl_world1_dp_step_equals_plain_step(attack):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(_free_port(), attack, q))
    p.start()
    res, tb = q.get(timeout=150)
    p.join(timeout=30)
    assert tb is None, tb
    assert res["backend"] == "nccl", res
    for sync_bn in (False, True):
        r = res[sync_bn]
        assert r["reducer"], r
        assert r["bn_calls"] == (6 * 4 if sync_bn else None), r
        assert r["params"] < 1e-6 and r["running"] < 1e-6 and r["nbt"], (sync_bn, r)
        assert r["loss"] < 1e-6 and r["acc"][0] == r["acc"][1] and r["samples"][0] == r["samples"][1], (sync_bn, r)
