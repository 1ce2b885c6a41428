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
    # metrics words: float64 loss sum (averaged) + counts (summed)
    m = torch.zeros(8, dtype=torch.int64)
    m[0:1] = torch.tensor([1.5 + rank], dtype=torch.float64).view(torch.int64)
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
    q.put((rank, torch.cat(allrows).tolist(), float(torch.abs(local - full).max()),
           float(red[0:1].view(torch.float64)), red[1:6].tolist(), berr))
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
    for rank, allrows, gerr, loss, cnt, berr in res:
        assert berr == 0.0                                    # bucketed == single all-reduce
        assert sorted(allrows) == list(range(64))            # disjoint cover of the epoch
        assert gerr < 1e-12                                   # sum of scaled shards == global mean grad
        assert loss == 2.0                                    # (1.5 + 2.5) / 2
        assert cnt == [16, 7, 4, 2, 4]
