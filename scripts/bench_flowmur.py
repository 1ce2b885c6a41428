#!/usr/bin/env python3
"""FlowMur trigger-optimisation throughput (utils/flowmur_generate_trigger.py:86-105 inner step).

One step = one batch of 256 clips (16 kHz x 1 s, resident in HBM): DEPLOY_CLAMP mix + MFCC,
frozen smallcnn eval forward + CE + input gradient, MFCC backward to the trigger, epoch-sum
accumulate, Adam, clamp.  Prints one JSON line (utterances/s) with the float64 oracle timed
on a small sample beside it.
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--cpu-sample", type=int, default=8)
    args = ap.parse_args()
    import numpy as np
    import torch
    import abd_amd
    from abd_amd import flowmur as FM, synth
    from abd_amd.models import smallcnn
    from golden_inputs import make_state
    abd_amd.load_library()
    dev = torch.device("cuda", 0)
    B, L, Lt = args.batch, 16000, 8000
    waves, _ = synth.make_clips_torch(B * 4, 16000, L, 10, seed=3, device=dev)
    st = make_state(32, 13, 10, 224, seed=9, trained_bn=True)
    m = smallcnn(10, 224)
    m.load_state_dict({k: torch.tensor(v) for k, v in st.items()})
    m = m.to(dev).eval()
    opt = FM.TriggerOptimizer(m, Lt)
    r = np.random.Generator(np.random.PCG64(0))
    labels = torch.full((B,), 2, dtype=torch.int64, device=dev)
    pos = [r.integers(0, L - Lt + 1, B) for _ in range(4)]
    for i in range(args.warmup):
        opt.step(waves[(i % 4) * B:(i % 4 + 1) * B], labels, pos[i % 4])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        opt.step(waves[(i % 4) * B:(i % 4 + 1) * B], labels, pos[i % 4])
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    # CPU baseline: the float64 oracle port on a small sample of the same step
    from oracle import flowmur as of, smallcnn as oc
    n = args.cpu_sample
    w = waves[:n].cpu().numpy().astype(np.float64)
    t1 = time.perf_counter()
    of.trigger_grad(oc.SmallCNN(st), w, np.full(Lt, 0.1), pos[0][:n], np.full(n, 2))
    cdt = time.perf_counter() - t1
    print(json.dumps({"metric": "FlowMur trigger-optimisation utterances/s (generate_trigger inner step)",
                      "value": round(B * args.steps / dt, 1), "unit": "utterances/s",
                      "ms_per_step": round(dt / args.steps * 1e3, 3), "batch": B, "steps": args.steps,
                      "dtype": "f32", "data": "synthetic",
                      "cpu_baseline": {"value": round(n / cdt, 2), "unit": "utterances/s", "cores": 1, "kind": "port",
                                       "sample": f"{n} clips, float64 numpy oracle, {cdt:.2f} s"}}), flush=True)


if __name__ == "__main__":
    main()
