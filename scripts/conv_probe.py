#!/usr/bin/env python3
"""Per-launch times of the smallcnn train-step kernels at the bench geometry (ultrasonic 100 x 40,
K = 35, B = 512) for one libabd build (ABD_LIB selects it): HIP-event phases over N train steps.

    ABD_LIB=.../libabd_x.so python scripts/conv_probe.py [--prec f32split] [--steps 30] [--tag x]
"""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--prec", default="f32split")
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--geom", default="100x40x35")
    ap.add_argument("--tag", default=os.path.basename(os.environ.get("ABD_LIB", "libabd.so")))
    args = ap.parse_args()
    import torch
    import abd_amd
    from abd_amd import _lib as L, training as T
    from abd_amd.models import smallcnn, geometry
    abd_amd.load_library()
    H, W, K = (int(v) for v in args.geom.split("x"))
    dev = torch.device("cuda", 0)
    torch.manual_seed(1)
    m = smallcnn(K, geometry(H, W)).to(dev).set_gemm_precision(args.prec)
    opt = torch.optim.Adam(m.parameters(), lr=1e-4)
    B = args.batch
    x = torch.randn(B, 1, H, W, device=dev) * 20
    y = torch.randint(0, K, (B,), device=dev)
    ind = (torch.rand(B, device=dev) < 0.1).long()
    m.train()
    eng = m.engine(x)
    adam = T.AdamBinding(m, opt)
    met = torch.zeros(L.METRICS_WORDS, dtype=torch.int64, device=dev)
    for _ in range(5):
        T.train_step(m, x, y, ind, adam, met)
    torch.cuda.synchronize()
    with L.PhaseProfiler(L.PHASES, max_records=64 * args.steps) as p:
        for _ in range(args.steps):
            T.train_step(m, x, y, ind, adam, met)
        torch.cuda.synchronize()
    ms = {k: round(v[0] / max(v[1], 1), 4) for k, v in p.result.items()}
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(args.steps):
        T.train_step(m, x, y, ind, adam, met)
    ev1.record()
    torch.cuda.synchronize()
    print(json.dumps({"tag": args.tag, "prec": args.prec, "geom": args.geom, "batch": B,
                      "step_ms": round(ev0.elapsed_time(ev1) / args.steps, 4), "phases": ms}), flush=True)


if __name__ == "__main__":
    main()
