"""GPU: FlowMur trigger optimisation sharded over 2 ranks (gloo, one GPU) == one process on the whole batch."""
import os
import socket

import numpy as np
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


def _run(world, rank, port, q):
    try:
        import sys
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        sys.path.insert(0, root)
        sys.path.insert(0, os.path.join(root, "tests"))
        import torch.distributed as dist
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        if world > 1:
            os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
            dist.init_process_group("gloo", rank=rank, world_size=world)
        import abd_amd
        from abd_amd import flowmur as FM, synth
        from abd_amd.models import smallcnn
        from golden_inputs import make_state
        abd_amd.load_library()
        st = make_state(32, 13, 10, 224, seed=9, trained_bn=True)
        m = smallcnn(10, 224)
        m.load_state_dict({k: torch.tensor(v) for k, v in st.items()})
        m = m.to(dev).eval()
        opt = FM.TriggerOptimizer(m, 8000)
        waves, _ = synth.make_clips_torch(64, 16000, 16000, 10, seed=3, device=dev)
        labels = torch.full((32,), 2, dtype=torch.int64, device=dev)
        r = np.random.default_rng(0)
        opt.new_epoch()
        for i in range(3):
            opt.step(waves[(i % 2) * 32:(i % 2 + 1) * 32], labels, r.integers(0, 8001, 32))
        loss = opt.epoch_loss()
        q.put((rank, opt.trigger.cpu().numpy(), loss, None))
        if world > 1:
            dist.destroy_process_group()
    except Exception:
        import traceback
        q.put((rank, None, None, traceback.format_exc()))
        raise


def test_trigger_optimisation_sharded_equals_single_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    p1 = ctx.Process(target=_run, args=(1, 0, port, q))
    p1.start()
    single = q.get(timeout=100)
    p1.join(timeout=30)
    ps = [ctx.Process(target=_run, args=(2, r, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=100) for _ in ps]
    for p in ps:
        p.join(timeout=30)
    assert single[3] is None, single[3]
    for rank, trig, loss, tb in res:
        assert tb is None, tb
        # Adam normalises the step, so trigger entries move by ~lr each step: compare at 1e-6 abs
        assert np.abs(trig - single[1]).max() < 1e-6
        assert abs(loss - single[2]) < 1e-5 * abs(single[2])
