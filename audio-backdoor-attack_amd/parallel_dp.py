"""Data-parallel plumbing (one process per GPU, torch.distributed; RCCL on the GPU box, gloo on CPU).

The path shards by utterance: every rank draws the same seeded epoch permutation and
takes its contiguous slice of each global batch; the only exchange is ONE sum
all-reduce of the flat fp32 gradient buffer per step (1.68 MB at 101x40),
with the loss gradient pre-normalised by the GLOBAL batch inside the loss kernel
(grad_scale = B_local / B_global), so the summed gradient is the global-batch mean.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_slice(pos: int, local_batch: int, rank: int, world: int):
    """[start, stop) of this rank's rows in the global batch that begins at epoch offset ``pos``."""
    s = pos + rank * local_batch
    return s, s + local_batch


def grad_scale(local_batch: int, global_batch: int) -> float:
    return float(local_batch) / float(global_batch)


def allreduce_grads(flat: torch.Tensor, group=None):
    """Sum the flat gradient buffer over ranks (one collective per step)."""
    dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)
    return flat


class OverlappedGradAllReduce:
    """Two-bucket gradient all-reduce overlapped with the conv backward.

    The flat gradient buffer is laid out conv1..bn3 then fc1/fc2; the fc tail (94 % of the
    bytes at 101x40) is final right after the fc1 weight-grad reduction, where libabd records
    ``event`` mid-backward (abd_train_args.fc_grads_event).  ``launch_fc`` makes a side stream
    wait for that event and starts the fc all-reduce there, so it runs over xGMI while the
    compute stream does the conv3/conv2/conv1 backward; ``finish`` all-reduces the small conv
    head on the compute stream and joins both before Adam.  No host synchronisation: with
    RCCL, ``Work.wait()`` only makes the current stream wait on the collective.
    """

    def __init__(self, flat: torch.Tensor, split: int, group=None):
        self.flat, self.split, self.group = flat, int(split), group
        self.head, self.tail = flat[:self.split], flat[self.split:]
        self.on_device = flat.is_cuda
        self._work = None
        if self.on_device:
            self.side = torch.cuda.Stream(flat.device)
            self.event = torch.cuda.Event()
            self.event.record()  # materialise the hipEvent handle libabd records into
        else:
            self.side = self.event = None

    def event_ptr(self):
        return self.event.cuda_event if self.event is not None else None

    def launch_fc(self):
        if self.on_device:
            self.side.wait_event(self.event)
            with torch.cuda.stream(self.side):
                self._work = dist.all_reduce(self.tail, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        else:
            self._work = dist.all_reduce(self.tail, op=dist.ReduceOp.SUM, group=self.group, async_op=True)

    def finish(self):
        w2 = dist.all_reduce(self.head, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        if self._work is not None:
            self._work.wait()
            self._work = None
        w2.wait()
        return self.flat


def broadcast_state(tensors, src: int = 0, group=None):
    """Make every rank start from (or return to) rank src's model state: the flat parameter
    buffer and the packed BN running statistics (DDP's init broadcast + broadcast_buffers)."""
    for t in tensors:
        if t is not None:
            dist.broadcast(t, src=src, group=group)


class SyncBatchNorm:
    """Synchronised BatchNorm statistics for the fused train step (abd_train_args.bn_sync*).

    The reference normalises over its whole batch (utils/models.py:20-30 in train mode); with
    per-rank statistics an N-GPU step differs from the 1-process step on the same global batch.
    libabd calls ``_sync`` six times per step (3 forward statistic reductions, 3 backward) with
    this rank's per-channel double sums (2C+1 values: sums, sums of squares / products, element
    count) written into ``buf``; the callback sums them over ranks with an all-reduce enqueued on
    the current stream (RCCL on the GPU box, gloo in rehearsals), and the kernels that follow use
    the global sums and count.  129 doubles per call: latency-bound, ~6 x 10 us on xGMI.
    """

    def __init__(self, device, group=None):
        from . import _lib as L
        self.group = group
        self.buf = torch.zeros(6 * L.BN_SYNC_STRIDE, dtype=torch.float64, device=device)
        self.calls = 0
        self.error = None

        def _sync(ctx, point, offset, n):
            try:
                dist.all_reduce(self.buf[offset:offset + n], op=dist.ReduceOp.SUM, group=self.group)
                self.calls += 1
                return 0
            except Exception as e:  # surfaced as an AbdError by the launch's return code
                self.error = e
                return 1

        self._cb = L.BN_SYNC_FN(_sync)   # keep the ctypes thunk alive as long as this object
        import ctypes as C
        self._cb_ptr = C.cast(self._cb, C.c_void_p).value

    def bind(self, args):
        args.bn_sync_buf = self.buf.data_ptr()
        args.bn_sync = self._cb_ptr
        args.bn_sync_ctx = None


def reduce_metrics(m: torch.Tensor, group=None) -> torch.Tensor:
    """Combine libabd metric words across ranks: counts summed, batch-mean loss averaged.

    Word 0 holds a float64 (sum of per-batch mean losses); words 1-5 are int64 counts."""
    out = m.clone()
    loss = out[0:1].view(torch.float64).clone()
    dist.all_reduce(loss, group=group)
    world = dist.get_world_size(group)
    loss /= world
    cnt = out[1:6].clone()
    dist.all_reduce(cnt, group=group)
    out[1:5] = cnt[0:4]
    out[5] = cnt[4] // world  # batches: every rank saw the same number of global batches
    out[0:1] = loss.view(torch.int64)
    return out
