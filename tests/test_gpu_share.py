"""GPU: two processes on one GPU repeat the same train step bit for bit.

With packed FP32 in the device code, kernels whose v_pk_fma_f32 low lane selected the high dword
of a source (conv1_stats_fold_kernel, conv1_wgrad_kernel) returned wrong low-lane values now and
then while another process shared the GPU (scripts/pk_opsel_probe.hip).  The
library is built without packed FP32 (tests/test_isa_cpu.py checks the code object); here two
processes each run the same f32split step (fixed inputs, masks and parameters, do_update=False)
ITERS times and every named workspace buffer and the gradients must equal the first repetition.
This is the layout of the 2-rank tests (test_gpu_dp.py, test_gpu_flowmur_dp.py)."""
import os
import sys

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
ITERS = 40
ORDER = ["coef", "p1", "r2", "p2", "r3", "xh3", "p3d", "d2", "logp", "dz", "rowinfo", "da", "dp3", "dz3",
         "dp2", "dz2", "bcoef", "dp1"]


def _worker(rank, q):
    try:
        sys.path.insert(0, ROOT)
        import abd_amd
        from abd_amd import training as T, models as M, _lib as L
        from abd_amd.models import smallcnn
        abd_amd.load_library()
        dev = torch.device("cuda", 0)
        B, H, W, K = 32, 101, 40, 10
        lf = M.geometry(H, W)
        g = torch.Generator(device="cpu").manual_seed(3 + rank)
        torch.manual_seed(35)
        m = smallcnn(K, lf).to(dev).set_gemm_precision("f32split").train()
        opt = torch.optim.Adam(m.parameters(), lr=1e-4)
        x = (torch.randn(B, 1, H, W, generator=g) * 20).to(dev)
        y = torch.randint(0, K, (B,), generator=g).to(dev)
        m1 = (torch.rand((B, lf), generator=g) < 0.6).to(torch.uint8).to(dev)
        m2 = (torch.rand((B, 128), generator=g) < 0.5).to(torch.uint8).to(dev)
        eng = m.engine(x)
        adam = T.AdamBinding(m, opt)
        ws = eng.workspace(B)
        offs = {n: L.lib().abd_smallcnn_workspace_offset(eng.h, B, n.encode()) for n in ORDER}
        offs = {n: o for n, o in offs.items() if o >= 0}
        ends = sorted(set(offs.values()) | {ws.numel()})
        region = {n: (o, min(e for e in ends if e > o)) for n, o in offs.items()}
        ref, bad = None, []
        for it in range(ITERS):
            eng.grads.fill_(1e30)
            T.train_step(m, x, y, None, adam, None, m1, m2, do_update=False, seed=1)
            torch.cuda.synchronize()
            snap = {n: ws[a:b].clone() for n, (a, b) in region.items()}
            snap["grads"] = eng.grads.clone()
            if ref is None:
                ref = snap
                continue
            diff = [n for n in snap if not torch.equal(snap[n], ref[n])]
            if diff:
                bad.append((it, diff))
        q.put((rank, bad, None))
    except Exception:
        import traceback
        q.put((rank, None, traceback.format_exc()))


def test_two_processes_repeat_the_step_bit_for_bit():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=110) for _ in ps]
    for p in ps:
        p.join(timeout=30)
    for rank, bad, tb in res:
        assert tb is None, tb
        assert not bad, (rank, bad[:3])
