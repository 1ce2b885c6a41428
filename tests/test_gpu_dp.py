"""GPU: the data-parallel step with the fc-gradient all-reduce overlapped with the conv backward.

Two ranks share the one GPU of the test box over gloo (RCCL needs one GPU per rank; the
8-GPU node runs the same code over RCCL).  Each rank computes its shard's gradients alone,
all-gathers them and sums (the expected result), then re-runs the same step through
ResidentTrainer's overlapped path (abd_train_args.fc_grads_event -> side-stream all-reduce
of the fc tail, conv head all-reduce, join) on a gradient buffer pre-filled with a sentinel,
so a collective that started before libabd wrote the fc gradients would show up.
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


def _worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        import sys
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        sys.path.insert(0, root)
        import torch.distributed as dist
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import abd_amd
        from abd_amd import features as F, synth, training as T
        from abd_amd.models import smallcnn
        from abd_amd.pipeline import ResidentTrainer, attack_config
        abd_amd.load_library()
        cfg = attack_config("badnets")
        B, K = 32, 10
        waves, labels = synth.make_clips_torch(128, cfg.sample_rate, cfg.length, K, seed=35 + rank, device=dev)
        torch.manual_seed(35)
        model = smallcnn(K, cfg.linear_features).to(dev)
        opt = torch.optim.Adam(model.parameters(), lr=1e-4)
        tr = ResidentTrainer(cfg, waves, labels, model, opt, B, seed=35, rank=rank, world=world)
        eng = model._engine
        g = torch.Generator(device="cpu")
        g.manual_seed(7 + rank)
        errs = []
        for step in range(3):
            rows = torch.arange(step * B, (step + 1) * B, dtype=torch.int32, device=dev)
            x = F.mfcc_batch(waves, tr.mcfg, rows=rows)
            y = labels[rows.long()].to(dev, torch.int64)
            ind = torch.zeros(B, dtype=torch.int64, device=dev)
            m1 = (torch.rand((B, eng.flat), generator=g) < 0.6).to(torch.uint8).to(dev)
            m2 = (torch.rand((B, 128), generator=g) < 0.5).to(torch.uint8).to(dev)
            scale = 1.0 / world
            T.train_step(model, x, y, ind, tr.adam, None, m1, m2, do_update=False, grad_scale=scale, seed=1)
            torch.cuda.synchronize()
            local = eng.grads.clone()
            parts = [torch.zeros_like(local) for _ in range(world)]
            dist.all_gather(parts, local)
            expect = torch.stack(parts).sum(0)
            eng.grads.fill_(1e30)
            T.train_step(model, x, y, ind, tr.adam, None, m1, m2, do_update=False, grad_scale=scale, seed=1,
                         fc_grads_event=tr.reducer.event_ptr())
            tr.reducer.launch_fc()
            tr.reducer.finish()
            T.apply_adam(model, tr.adam, dev)
            torch.cuda.synchronize()
            errs.append(float(((eng.grads - expect).abs() / (expect.abs() + 1e-6)).max()))
        p = eng.params.clone()
        parts = [torch.zeros_like(p) for _ in range(world)]
        dist.all_gather(parts, p)
        same = float((parts[0] - parts[1]).abs().max())
        q.put((rank, errs, same, None))
        dist.destroy_process_group()
    except Exception as e:  # report instead of hanging the parent
        import traceback
        q.put((rank, None, None, traceback.format_exc()))
        raise


def test_overlapped_allreduce_matches_gathered_sum():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=110) for _ in ps]
    for p in ps:
        p.join(timeout=30)
    for rank, errs, same, tb in res:
        assert tb is None, tb
        assert max(errs) < 1e-6, errs          # overlapped buckets == sum of the shards' gradients
        assert same == 0.0                     # identical Adam updates on every rank


def _equiv_worker(rank, world, port, q):
    """2 ranks x B/2 with synchronised BatchNorm vs 1 rank x B, same global batches."""
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        import sys
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        sys.path.insert(0, root)
        import torch.distributed as dist
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import abd_amd
        from abd_amd import synth, training as T
        from abd_amd.models import smallcnn
        from abd_amd.pipeline import ResidentTrainer, attack_config
        abd_amd.load_library()
        cfg = attack_config("badnets")
        B, K, steps = 64, 10, 3
        waves, labels = synth.make_clips_torch(256, cfg.sample_rate, cfg.length, K, seed=35, device=dev)

        # the 1-rank reference runs the same data-parallel code path (SyncBN over a one-rank group:
        # no BN1 fold, the activation passes for the BN sums, the unfused fc head): the fused
        # single-rank path differs from it in fp32 rounding, which Adam's sign-like first steps turn
        # into +-lr parameter differences
        solo = dist.new_group([0])

        def run(world_, rank_, pg_world):
            # rank 1 seeded differently (the seed + rank pattern): parameters, BN buffers AND the
            # dropout seed come from rank 0, so the run still equals the 1-rank run
            torch.manual_seed(35 + 1000 * rank_)
            model = smallcnn(K, cfg.linear_features).to(dev)
            opt = torch.optim.Adam(model.parameters(), lr=1e-3)
            tr = ResidentTrainer(cfg, waves, labels, model, opt, B // world_, seed=35, rank=rank_, world=world_,
                                 sync_bn=True, collectives=True, process_group=None if world_ > 1 else solo)
            for _ in range(steps):
                tr.step()
            m = tr.read_metrics()
            eng = model._engine
            torch.cuda.synchronize()
            return eng.params.clone(), eng.running.clone(), m, tr

        p2, r2, m2, tr2 = run(world, rank, world)
        assert tr2.bn_sync is not None and tr2.bn_sync.calls == 6 * steps, tr2.bn_sync.calls
        # dropout masks of the two ranks hash their GLOBAL rows: rank 1 must not repeat rank 0's
        eng = tr2.model._engine
        x = torch.zeros((B // world, 1, tr2.T, cfg.n_mfcc), device=dev)
        mo = (torch.empty((B // world, eng.flat), dtype=torch.uint8, device=dev),
              torch.empty((B // world, 128), dtype=torch.uint8, device=dev))
        T.train_step(tr2.model, x, torch.zeros(B // world, dtype=torch.int64, device=dev), None, None, None,
                     masks_out=mo, do_update=False, seed=9, row_offset=rank * (B // world))
        parts = [torch.zeros_like(mo[0]) for _ in range(world)]
        dist.all_gather(parts, mo[0])
        masks_differ = not torch.equal(parts[0], parts[1])
        res = None
        if rank == 0:
            p1, r1, m1, _ = run(1, 0, 1)
            nrel = lambda a, b: float((a - b).norm() / b.norm())  # noqa: E731
            res = {"params": nrel(p2, p1), "running": nrel(r2, r1), "loss": abs(m2["loss"] - m1["loss"]) / m1["loss"],
                   "acc": (m2["acc"], m1["acc"]), "samples": (m2["samples"], m1["samples"])}
        q.put((rank, res, masks_differ, None))
        dist.destroy_process_group()
    except Exception:
        import traceback
        q.put((rank, None, None, traceback.format_exc()))
        raise


def test_two_rank_sync_bn_step_equals_one_rank_step():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_equiv_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=110) for _ in ps]
    for p in ps:
        p.join(timeout=30)
    for rank, r, differ, tb in res:
        assert tb is None, tb
        assert differ, "ranks drew identical dropout masks"
        if rank == 0:
            assert r["params"] < 1e-5 and r["running"] < 1e-5, r
            assert r["loss"] < 1e-5 and r["acc"][0] == r["acc"][1] and r["samples"][0] == r["samples"][1], r


def _tail_worker(rank, world, port, q, N):
    """A full epoch of N rows (not a multiple of the global batch) on the daba geometry (32x40 Slaney
    front end, fc 896): 2 ranks x 32 with SyncBN vs 1 rank x 64; the last batch is kept
    (drop_last=False, daba.py:152-154) and split unevenly -- for N % 64 == 1 rank 1 has no rows."""
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        import sys
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        sys.path.insert(0, root)
        import torch.distributed as dist
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import abd_amd
        from abd_amd import synth
        from abd_amd.models import smallcnn
        from abd_amd.pipeline import ResidentTrainer, attack_config
        abd_amd.load_library()
        cfg = attack_config("daba")
        G, K = 64, 10
        waves, labels = synth.make_clips_torch(N, cfg.sample_rate, cfg.length, K, seed=36, device=dev)

        solo = dist.new_group([0])   # the 1-rank reference on the same (SyncBN) code path

        def run(world_, rank_):
            torch.manual_seed(35)
            model = smallcnn(K, cfg.linear_features).to(dev)
            opt = torch.optim.Adam(model.parameters(), lr=1e-3)
            tr = ResidentTrainer(cfg, waves, labels, model, opt, G // world_, seed=35, rank=rank_, world=world_,
                                 sync_bn=True, collectives=True, process_group=None if world_ > 1 else solo)
            steps = tr.steps_per_epoch()
            m = tr.run_epoch()
            tr.sync_buffers()
            eng = model._engine
            torch.cuda.synchronize()
            return eng.params.clone(), eng.running.clone(), eng.nbt.clone(), m, steps, tr.adam.step

        p2, r2, n2, m2, steps2, adam2 = run(world, rank)
        res = None
        if rank == 0:
            p1, r1, n1, m1, steps1, adam1 = run(1, 0)
            nrel = lambda a, b: float((a - b).norm() / b.norm())  # noqa: E731
            res = {"params": nrel(p2, p1), "running": nrel(r2, r1), "nbt": (n2.tolist(), n1.tolist()),
                   "loss": abs(m2["loss"] - m1["loss"]) / m1["loss"], "acc": (m2["acc"], m1["acc"]),
                   "samples": (m2["samples"], m1["samples"]), "steps": (steps2, steps1), "adam": (adam2, adam1)}
        q.put((rank, res, None))
        dist.destroy_process_group()
    except Exception:
        import traceback
        q.put((rank, None, traceback.format_exc()))
        raise


@pytest.mark.parametrize("N", [230, 193])
def test_two_rank_uneven_tail_epoch_equals_one_rank(N):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_tail_worker, args=(r, 2, port, q, N)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=110) for _ in ps]
    for p in ps:
        p.join(timeout=30)
    for rank, r, tb in res:
        assert tb is None, tb
        if rank == 0:
            assert r["steps"] == (4, 4) and r["adam"] == (4, 4), r
            assert r["samples"] == (N, N), r
            assert r["params"] < 1e-5 and r["running"] < 1e-5 and r["loss"] < 1e-5, r
            assert r["acc"][0] == r["acc"][1] and r["nbt"][0] == r["nbt"][1], r


def _syncbn_grad_worker(port, q):
    """the SyncBN step's code path (no BN1 fold, BN sums from activation passes, the
    unfused fc head) against the plain fused single-rank step, one step, do_update=False -- no Adam
    amplification, so the two agree to fp32 rounding."""
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        import sys
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        sys.path.insert(0, root)
        import torch.distributed as dist
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        dist.init_process_group("gloo", rank=0, world_size=1)
        import abd_amd
        from abd_amd import features as F, models as M, parallel_dp as DP, synth, training as T
        from abd_amd.models import smallcnn
        from abd_amd.pipeline import attack_config
        abd_amd.load_library()
        out = {}
        for name, prec in (("badnets", "f32split"), ("badnets", "f32"), ("daba", "f32split")):
            cfg = attack_config(name)
            B, K = 48, 10
            waves, labels = synth.make_clips_torch(B, cfg.sample_rate, cfg.length, K, seed=41, device=dev)
            torch.manual_seed(35)
            model = smallcnn(K, cfg.linear_features).to(dev).set_gemm_precision(prec)
            opt = torch.optim.Adam(model.parameters(), lr=1e-4)
            x = F.mfcc_batch(waves, cfg.mfcc(), rows=torch.arange(B, dtype=torch.int32, device=dev))
            y = labels.to(dev, torch.int64)
            ind = torch.zeros(B, dtype=torch.int64, device=dev)
            eng = model.engine(x)
            adam = T.AdamBinding(model, opt)
            g = torch.Generator(device="cpu").manual_seed(5)
            m1 = (torch.rand((B, eng.flat), generator=g) < 0.6).to(torch.uint8).to(dev)
            m2 = (torch.rand((B, 128), generator=g) < 0.5).to(torch.uint8).to(dev)
            run0 = eng.running.clone()
            res = []
            for sync in (None, DP.SyncBatchNorm(dev)):
                eng.running.copy_(run0)
                eng.grads.fill_(1e30)
                T.train_step(model, x, y, ind, adam, None, m1, m2, do_update=False, seed=1, bn_sync=sync)
                torch.cuda.synchronize()
                res.append((eng.grads.clone(), eng.running.clone(), None if sync is None else sync.calls))
            (ga, ra, _), (gb, rb, calls) = res
            per = {p: float((u - v).norm() / max(float(v.norm()), 1e-30))
                   for p, u, v in zip(M.PARAM_ORDER, eng.views(gb), eng.views(ga))}
            out[(name, prec)] = {"calls": calls, "grads": per,
                                 "running": float((rb - ra).norm() / (ra - run0).norm())}
        q.put((out, None))
        dist.destroy_process_group()
    except Exception:
        import traceback
        q.put((None, traceback.format_exc()))
        raise


def test_world1_sync_bn_gradients_equal_fused_step():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_syncbn_grad_worker, args=(_free_port(), q))
    p.start()
    out, tb = q.get(timeout=110)
    p.join(timeout=30)
    assert tb is None, tb
    for key, r in out.items():
        print(key, r["calls"], f"running {r['running']:.1e}", {k: f"{v:.1e}" for k, v in r["grads"].items()})
        assert r["calls"] == 6, (key, r["calls"])             # the SyncBN path really ran
        assert r["running"] < 1e-5, (key, r)                  # BN batch statistics (running-stat update)
        for pname, e in r["grads"].items():
            assert e < 1e-5, (key, pname, e)                  # every parameter gradient
