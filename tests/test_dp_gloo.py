"""CPU: the data-parallel plumbing with world_size 2 over gloo (the GPU box uses RCCL)."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import abd_amd  # noqa: F401
    from abd_amd import parallel_dp as DP
    N, B = 64, 8
    g = torch.Generator()
    g.manual_seed(35)
    perm = torch.randperm(N, generator=g)  # identical on every rank
    rows = []
    for step in range(N // (B * world)):
        s, e = DP.shard_slice(step * B * world, B, rank, world)
        rows.append(perm[s:e])
    rows = torch.cat(rows)
    allrows = [torch.zeros_like(rows) for _ in range(world)]
    dist.all_gather(allrows, rows)
    # gradient convention: per-row contributions scaled by 1/B_global, summed over ranks
    r = np.random.default_rng(0)
    feats = torch.tensor(r.standard_normal((N, 5)))
    dlog = torch.tensor(r.standard_normal((N, 3)))
    mine = perm[rank * B:(rank + 1) * B]
    local = (dlog[mine] * DP.grad_scale(B, B * world) / B).T @ feats[mine]
    DP.allreduce_grads(local)
    glob_rows = perm[:B * world]
    full = (dlog[glob_rows] / (B * world)).T @ feats[glob_rows]
    # metrics words: float64 loss sums (each rank's batch means weighted by B_local / B_global,
    # so they are summed) + counts (summed)
    m = torch.zeros(8, dtype=torch.int64)
    m[0:1] = torch.tensor([(1.5 + rank) * DP.grad_scale(B, B * world)], dtype=torch.float64).view(torch.int64)
    m[1:6] = torch.tensor([B, 3 + rank, 2, 1, 4])
    red = DP.reduce_metrics(m)
    # two-bucket overlapped all-reduce == one all-reduce of the flat buffer
    flat = torch.tensor(r.standard_normal(1000) + rank)
    ref = flat.clone()
    DP.allreduce_grads(ref)
    red2 = DP.OverlappedGradAllReduce(flat, 937)
    assert red2.event_ptr() is None
    red2.launch_fc()
    red2.finish()
    berr = float(torch.abs(flat - ref).max())
    # uneven last batches (drop_last=False): floor/ceil shares cover the epoch exactly, and the
    # count-weighted shard gradients / losses sum to the global batch's mean
    tails = {}
    for n in (70, 65, 64 + 13):
        cover, gerr_t, lsum = [], 0.0, 0.0
        pos = 0
        while pos < n:
            gb = min(B * world, n - pos)
            s, e = DP.shard_range(pos, gb, rank, world)
            mine = torch.arange(s, e)
            cover.append(mine)
            loc = torch.zeros(3, 5, dtype=torch.float64)
            if e > s:
                loc = (dlog[mine % N] * DP.grad_scale(e - s, gb) / (e - s)).T @ feats[mine % N]
                lsum_r = float(dlog[mine % N, 0].mean()) * DP.grad_scale(e - s, gb)
            else:
                lsum_r = 0.0
            DP.allreduce_grads(loc)
            lt = torch.tensor([lsum_r], dtype=torch.float64)
            DP.allreduce_grads(lt)
            glob = torch.arange(pos, pos + gb)
            ref = (dlog[glob % N] / gb).T @ feats[glob % N]
            gerr_t = max(gerr_t, float(torch.abs(loc - ref).max()),
                         abs(float(lt) - float(dlog[glob % N, 0].mean())))
            pos += gb
        got = torch.cat(cover)
        sizes = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(sizes, torch.tensor([got.numel()]))
        allc = [torch.zeros(int(sz), dtype=torch.int64) for sz in sizes]
        if any(int(sz) != got.numel() for sz in sizes):
            padded = torch.full((max(int(sz) for sz in sizes),), -1, dtype=torch.int64)
            padded[:got.numel()] = got
            allc = [torch.zeros_like(padded) for _ in range(world)]
            dist.all_gather(allc, padded)
            allc = [a[a >= 0] for a in allc]
        else:
            dist.all_gather(allc, got)
        tails[n] = (sorted(torch.cat(allc).tolist()) == list(range(n)), gerr_t)
    # a rank without rows joins the SyncBatchNorm reductions with zeros
    sb = DP.SyncBatchNorm(torch.device("cpu"))
    sb.idle()
    q.put((rank, torch.cat(allrows).tolist(), float(torch.abs(local - full).max()),
           float(red[0:1].view(torch.float64)), red[1:6].tolist(), berr, tails, sb.calls,
           float(sb.buf.abs().sum())))
    dist.destroy_process_group()


def test_world2_sharding_gradients_and_metrics():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, allrows, gerr, loss, cnt, berr, tails, calls, bsum in res:
        assert all(ok and e < 1e-12 for ok, e in tails.values()), tails
        assert calls == 6 and bsum == 0.0
        assert berr == 0.0                                    # bucketed == single all-reduce
        assert sorted(allrows) == list(range(64))            # disjoint cover of the epoch
        assert gerr < 1e-12                                   # sum of scaled shards == global mean grad
        assert loss == 2.0                                    # 1.5 / 2 + 2.5 / 2
        assert cnt == [16, 7, 4, 2, 4]
