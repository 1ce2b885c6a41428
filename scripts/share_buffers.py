#!/usr/bin/env python3
"""Which train-step buffer first goes nondeterministic under GPU sharing: NPROC processes on one GPU
each repeat the same step (fixed inputs, masks, parameters; do_update=False) and compare every
named workspace buffer and the gradients with the first repetition, bit for bit.  Buffers are
listed in pipeline order, so the first one differing in an iteration is where it starts.
    python scripts/share_buffers.py PREC [NPROC] [ITERS] [B]"""
import os
import sys

import torch
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
ORDER = ["coef", "p1", "p1s", "r2", "p2", "r3", "xh3", "p3d", "d2", "logp", "dz", "rowinfo", "da", "dp3", "dz3",
         "dp2", "dz2", "dz2s", "bcoef", "dp1"]


def worker(rank, prec, iters, B, q):
    sys.path.insert(0, os.path.dirname(HERE))
    import abd_amd
    from abd_amd import training as T, models as M, _lib as L
    from abd_amd.models import smallcnn
    abd_amd.load_library()
    dev = torch.device("cuda", 0)
    H, W, K = 101, 40, 10
    lf = M.geometry(H, W)
    g = torch.Generator(device="cpu").manual_seed(3 + rank)
    torch.manual_seed(35)
    m = smallcnn(K, lf).to(dev).set_gemm_precision(prec).train()
    opt = torch.optim.Adam(m.parameters(), lr=1e-4)
    x = (torch.randn(B, 1, H, W, generator=g) * 20).to(dev)
    y = torch.randint(0, K, (B,), generator=g).to(dev)
    m1 = (torch.rand((B, lf), generator=g) < 0.6).to(torch.uint8).to(dev)
    m2 = (torch.rand((B, 128), generator=g) < 0.5).to(torch.uint8).to(dev)
    eng = m.engine(x)
    adam = T.AdamBinding(m, opt)
    ws = eng.workspace(B)
    offs = {}
    for n in ORDER:
        o = L.lib().abd_smallcnn_workspace_offset(eng.h, B, n.encode())
        if o >= 0:
            offs[n] = o
    ends = sorted(set(offs.values()) | {ws.numel()})
    region = {n: (o, min(e for e in ends if e > o)) for n, o in offs.items()}
    ref = None
    bad = []
    x0, p0 = x.clone(), eng.params.clone()
    for it in range(iters):
        eng.grads.fill_(1e30)
        T.train_step(m, x, y, None, adam, None, m1, m2, do_update=False, seed=1)
        torch.cuda.synchronize()
        snap = {n: ws[a:b].clone() for n, (a, b) in region.items()}
        snap["grads"] = eng.grads.clone()
        if ref is None:
            ref = snap
            continue
        diff = [n for n in ORDER + ["grads"] if n in snap and not torch.equal(snap[n], ref[n])]
        if not torch.equal(x, x0) or not torch.equal(eng.params, p0):
            diff.append("INPUTS-CHANGED")
        if diff:
            gd = [p for p, u, v in zip(M.PARAM_ORDER, eng.views(snap["grads"]), eng.views(ref["grads"]))
                  if not torch.equal(u, v)]
            detail = []
            for n in diff[:3]:
                if n not in snap:
                    continue
                u, v = snap[n].view(torch.int32), ref[n].view(torch.int32)
                idx = (u != v).nonzero().flatten()
                uf, vf = snap[n].view(torch.float32), ref[n].view(torch.float32)
                i0 = int(idx[0])
                detail.append((n, int(idx.numel()), int(u.numel()), i0, int(idx[-1]),
                               float(uf[i0]), float(vf[i0]), float((uf[idx] - vf[idx]).abs().max()),
                               int(region[n][0]) if n in region else -1))
            bad.append((it, diff, gd, detail))
            if os.environ.get("SUMMARY"):
                import collections
                summ = {}
                if "p1" in diff:
                    idx = (snap["p1"].view(torch.int32) != ref["p1"].view(torch.int32)).nonzero().flatten().cpu()
                    idx = idx[idx < B * 100 * 13 * 64]
                    c = idx % 64
                    pos = idx // 64
                    w = pos % 13
                    h = (pos // 13) % 100
                    b = pos // 1300
                    summ["p1_b_chunk"] = sorted(collections.Counter(zip(b.tolist(), (h // 8).tolist())).items())[:12]
                    summ["p1_c"] = sorted(collections.Counter(c.tolist()).items())[:64]
                    summ["p1_w"] = sorted(collections.Counter(w.tolist()).items())
                    summ["p1_hmod8"] = sorted(collections.Counter((h % 8).tolist()).items())
                if "dp1" in diff:
                    base = (51497984 - region["dp1"][0]) // 4
                    idx = (snap["dp1"].view(torch.int32) != ref["dp1"].view(torch.int32)).nonzero().flatten().cpu()
                    dp = idx[idx < B * 100 * 13 * 64]
                    summ["dp1_n"] = int(dp.numel())
                    pi = idx[(idx >= base) & (idx < base + 416 * 320)] - base
                    summ["part_blk"] = sorted(collections.Counter((pi % 416).tolist()).items())[:40]
                    summ["part_col"] = sorted(collections.Counter((pi // 416).tolist()).items())[:80]
                print("SUMMARY", rank, it, summ, flush=True)
    q.put((rank, prec, os.environ.get("ABD_WS_DMA", "1"), B, bad))


def main():
    prec = sys.argv[1]
    nproc = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    iters = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    B = int(sys.argv[4]) if len(sys.argv) > 4 else 32
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, prec, iters, B, q)) for r in range(nproc)]
    for p in ps:
        p.start()
    res = [q.get(timeout=150) for _ in ps]
    for p in ps:
        p.join(timeout=30)
    for r in sorted(res):
        print(r, flush=True)


if __name__ == "__main__":
    main()
