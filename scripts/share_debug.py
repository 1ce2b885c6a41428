#!/usr/bin/env python3
"""Determinism under GPU sharing: NPROC processes on one GPU each run the same train step twice
(do_update=False) per iteration and compare the gradients bit for bit -- no collectives at all.
    python scripts/share_debug.py PREC [NPROC] [ITERS]"""
import os
import sys

import torch
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))


def worker(rank, prec, iters, q):
    sys.path.insert(0, os.path.dirname(HERE))
    import abd_amd
    from abd_amd import training as T, models as M
    from abd_amd.models import smallcnn
    abd_amd.load_library()
    dev = torch.device("cuda", 0)
    H, W, K, B = 101, 40, 10, 32
    lf = M.geometry(H, W)
    g = torch.Generator(device="cpu").manual_seed(3 + rank)
    torch.manual_seed(35)
    m = smallcnn(K, lf).to(dev).set_gemm_precision(prec).train()
    opt = torch.optim.Adam(m.parameters(), lr=1e-4)
    x = (torch.randn(B, 1, H, W, generator=g) * 20).to(dev)
    eng = m.engine(x)
    adam = T.AdamBinding(m, opt)
    bad = []
    for it in range(iters):
        x = (torch.randn(B, 1, H, W, generator=g) * 20).to(dev)
        y = torch.randint(0, K, (B,), generator=g).to(dev)
        m1 = (torch.rand((B, lf), generator=g) < 0.6).to(torch.uint8).to(dev)
        m2 = (torch.rand((B, 128), generator=g) < 0.5).to(torch.uint8).to(dev)
        T.train_step(m, x, y, None, adam, None, m1, m2, do_update=False, seed=1)
        a = eng.grads.clone()
        eng.grads.fill_(1e30)
        T.train_step(m, x, y, None, adam, None, m1, m2, do_update=False, seed=1)
        b = eng.grads.clone()
        torch.cuda.synchronize()
        diff = [n for n, u, v in zip(M.PARAM_ORDER, eng.views(a), eng.views(b)) if not torch.equal(u, v)]
        if diff:
            bad.append((it, diff))
        T.apply_adam(m, adam, dev)
    q.put((rank, prec, os.environ.get("ABD_WS_DMA", "1"), bad))


def main():
    prec = sys.argv[1]
    nproc = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    iters = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, prec, iters, q)) for r in range(nproc)]
    for p in ps:
        p.start()
    res = [q.get(timeout=150) for _ in ps]
    for p in ps:
        p.join(timeout=30)
    for r in sorted(res):
        print(r, flush=True)


if __name__ == "__main__":
    main()
