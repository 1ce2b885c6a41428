#!/usr/bin/env python3
"""Debug probe: (1) per-parameter gradient differences of one train step with SyncBatchNorm over a
one-rank gloo group against the plain step, per GEMM precision; (2) the same step launched twice on
the same inputs and parameters (do_update=False) must give bit-identical gradients, over a few
iterations with Adam in between (state carried between launches would show up here)."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def main():
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=os.environ.get("PORT", "29561"))
    dist.init_process_group("gloo", rank=0, world_size=1)
    import abd_amd
    from abd_amd import training as T, parallel_dp as DP, models as M
    from abd_amd.models import smallcnn
    abd_amd.load_library()
    dev = torch.device("cuda", 0)
    H, W, K, B = int(os.environ.get("H", 101)), int(os.environ.get("W", 40)), 10, int(os.environ.get("B", 64))
    lf = M.geometry(H, W)
    g = torch.Generator(device="cpu").manual_seed(3)
    x = (torch.randn(B, 1, H, W, generator=g) * 20).to(dev)
    y = torch.randint(0, K, (B,), generator=g).to(dev)
    ind = (torch.rand(B, generator=g) < 0.2).long().to(dev)
    m1 = (torch.rand((B, lf), generator=g) < 0.6).to(torch.uint8).to(dev)
    m2 = (torch.rand((B, 128), generator=g) < 0.5).to(torch.uint8).to(dev)
    names = M.PARAM_ORDER
    allg = {}
    for prec in ("f32", "f32split", "bf16"):
        out = {}
        for sync in (False, True):
            torch.manual_seed(35)
            m = smallcnn(K, lf).to(dev).set_gemm_precision(prec).train()
            opt = torch.optim.Adam(m.parameters(), lr=1e-3)
            eng = m.engine(x)
            adam = T.AdamBinding(m, opt)
            sb = DP.SyncBatchNorm(dev) if sync else None
            T.train_step(m, x, y, ind, adam, None, m1, m2, do_update=False, seed=1, bn_sync=sb)
            torch.cuda.synchronize()
            out[sync] = [v.clone() for v in eng.views(eng.grads)]
        diffs = {n: float((a - b).norm() / max(float(b.norm()), 1e-30)) for n, a, b in zip(names, out[True], out[False])}
        print(prec, "sync vs plain grads:", " ".join(f"{n}={v:.1e}" for n, v in diffs.items()), flush=True)
        allg[prec] = out
    for prec in ("f32split", "bf16"):
        for sync in (False, True):
            diffs = {n: float((a - b).norm() / max(float(b.norm()), 1e-30))
                     for n, a, b in zip(names, allg[prec][sync], allg["f32"][sync])}
            print(prec, "vs f32", "sync" if sync else "plain", " ".join(f"{n}={v:.1e}" for n, v in diffs.items()),
                  flush=True)
    for prec in ("f32", "f32split"):
        torch.manual_seed(35)
        m = smallcnn(K, lf).to(dev).set_gemm_precision(prec).train()
        opt = torch.optim.Adam(m.parameters(), lr=1e-3)
        eng = m.engine(x)
        adam = T.AdamBinding(m, opt)
        res = []
        for it in range(4):
            T.train_step(m, x, y, ind, adam, None, m1, m2, do_update=False, seed=1)
            torch.cuda.synchronize()
            a = eng.grads.clone()
            eng.grads.fill_(1e30)
            T.train_step(m, x, y, ind, adam, None, m1, m2, do_update=False, seed=1)
            torch.cuda.synchronize()
            b = eng.grads.clone()
            bad = [n for n, u, v in zip(names, eng.views(a), eng.views(b)) if not torch.equal(u, v)]
            res.append(bad)
            T.apply_adam(m, adam, dev)
        print(prec, "repeat-launch differences per iteration:", res, flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
