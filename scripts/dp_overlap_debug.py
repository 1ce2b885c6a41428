#!/usr/bin/env python3
"""Debug probe for tests/test_gpu_dp.py::test_overlapped_allreduce_matches_gathered_sum: two gloo
ranks on one GPU, per-parameter worst relative error of the overlapped all-reduce per iteration."""
import os
import sys
import socket

import torch
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))


def worker(rank, world, port, prec, iters, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, os.path.dirname(HERE))
    import torch.distributed as dist
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import abd_amd
    from abd_amd import features as F, synth, training as T, models as M
    from abd_amd.models import smallcnn
    from abd_amd.pipeline import ResidentTrainer, attack_config
    abd_amd.load_library()
    cfg = attack_config("badnets")
    B, K = 32, 10
    waves, labels = synth.make_clips_torch(32 * iters, cfg.sample_rate, cfg.length, K, seed=35 + rank, device=dev)
    torch.manual_seed(35)
    model = smallcnn(K, cfg.linear_features).to(dev).set_gemm_precision(prec)
    opt = torch.optim.Adam(model.parameters(), lr=1e-4)
    tr = ResidentTrainer(cfg, waves, labels, model, opt, B, seed=35, rank=rank, world=world)
    eng = model._engine
    g = torch.Generator(device="cpu")
    g.manual_seed(7 + rank)
    out = []
    for step in range(iters):
        rows = torch.arange(step * B, (step + 1) * B, dtype=torch.int32, device=dev)
        x = F.mfcc_batch(waves, tr.mcfg, rows=rows)
        y = labels[rows.long()].to(dev, torch.int64)
        ind = torch.zeros(B, dtype=torch.int64, device=dev)
        m1 = (torch.rand((B, eng.flat), generator=g) < 0.6).to(torch.uint8).to(dev)
        m2 = (torch.rand((B, 128), generator=g) < 0.5).to(torch.uint8).to(dev)
        T.train_step(model, x, y, ind, tr.adam, None, m1, m2, do_update=False, grad_scale=0.5, seed=1)
        torch.cuda.synchronize()
        local = eng.grads.clone()
        parts = [torch.zeros_like(local) for _ in range(world)]
        dist.all_gather(parts, local)
        expect = torch.stack(parts).sum(0)
        eng.grads.fill_(1e30)
        T.train_step(model, x, y, ind, tr.adam, None, m1, m2, do_update=False, grad_scale=0.5, seed=1,
                     fc_grads_event=tr.reducer.event_ptr())
        tr.reducer.launch_fc()
        tr.reducer.finish()
        torch.cuda.synchronize()
        got = eng.grads.clone()
        T.apply_adam(model, tr.adam, dev)
        torch.cuda.synchronize()
        rel = (got - expect).abs() / (expect.abs() + 1e-6)
        worst = {}
        for n, v, e, gg, lc in zip(M.PARAM_ORDER, eng.views(rel), eng.views(expect), eng.views(got), eng.views(local)):
            if float(v.max()) > 1e-6:
                i = int(v.argmax())
                worst[n] = (float(v.max()), float(e[i]), float(gg[i]), float(lc[i]), int((v > 1e-6).sum()))
        out.append(worst)
    q.put((rank, prec, out))
    dist.destroy_process_group()


def main():
    ctx = mp.get_context("spawn")
    for prec in sys.argv[1:] or ["f32", "f32split"]:
        for rep in range(2):
            q = ctx.Queue()
            s = socket.socket()
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
            s.close()
            ps = [ctx.Process(target=worker, args=(r, 2, port, prec, 5, q)) for r in range(2)]
            for p in ps:
                p.start()
            res = [q.get(timeout=120) for _ in ps]
            for p in ps:
                p.join(timeout=30)
            for rank, pr, out in sorted(res):
                print(pr, "rep", rep, "rank", rank, [(i, w) for i, w in enumerate(out) if w], flush=True)


if __name__ == "__main__":
    main()
