#!/usr/bin/env python3
"""Secondary measurements: every BASELINE.json config's per-batch hot path at N=1, plus the
offline stages the reference runs once per clip (DABA selection, JingleBack styling, resampling).

One JSON line per workload on stdout.  bench.py stays the headline (configs[1]); this script
backs the per-config numbers in DESIGN.md.  Synthetic 16 kHz / 44.1 kHz clips resident in HBM.

    python scripts/bench_configs.py [--steps 20]
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)


def timed(fn, steps, warmup=3):
    import torch
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--only", default="")
    ap.add_argument("--fp32-mode", default="f32split", choices=("f32split", "f32"),
                    help="conv GEMMs of the fp32 configs (f32split = bench.py's default, fp32-accurate)")
    args = ap.parse_args()
    import numpy as np
    import torch
    import abd_amd
    from abd_amd import synth, features as F, daba as D, triggers as TR
    from abd_amd.models import smallcnn
    from abd_amd.pipeline import ResidentTrainer, attack_config, ultrasonic_trigger
    abd_amd.load_library()
    dev = torch.device("cuda", 0)
    only = set(args.only.split(",")) if args.only else None

    def emit(d):
        print(json.dumps(d), flush=True)

    # ---- training step per attack (BASELINE configs[0..4] at one GPU)
    FP = args.fp32_mode
    plan = [("badnets", 10, 256, FP, "configs[0] badnets.py (GPU form of the CPU-only reference config)"),
            ("ultrasonic", 35, 512, FP, "configs[1] ultrasonic.py (headline; bench.py)"),
            ("ultrasonic", 35, 512, "bf16", "configs[1] shape with bf16 conv GEMMs (not the headline: fp32 parity)"),
            ("jingleback", 10, 256, FP, "configs[2] jingleback.py style 5, fp32-accurate GEMMs"),
            ("jingleback", 10, 256, "bf16", "configs[2] jingleback.py style 5, bf16 conv GEMMs on MFMA (the config's dtype)"),
            ("daba", 10, 256, FP, "configs[3] daba.py training step (librosa 32x40 features)"),
            ("flowmur", 10, 256, FP, "configs[4] flowmur.py poisoned training (smallcnn 32x13)")]
    for name, K, B, prec, what in plan:
        if only and name not in only:
            continue
        cfg = attack_config(name)
        N = 4096
        waves, labels = synth.make_clips_torch(N, cfg.sample_rate, cfg.length, K, seed=5, device=dev)
        trig = None
        if name == "ultrasonic":
            trig = ultrasonic_trigger(60, "mid", False)
        elif name == "flowmur":
            trig = (0.05 * np.random.default_rng(1).standard_normal(8000)).astype(np.float32)
        torch.manual_seed(35)
        model = smallcnn(K, cfg.linear_features).to(dev)
        opt = torch.optim.Adam(model.parameters(), lr=1e-4)
        tr = ResidentTrainer(cfg, waves, labels, model, opt, B, trigger=trig, seed=35, gemm_precision=prec)
        dt = timed(tr.step, args.steps)
        emit({"workload": f"train_step:{name}", "what": what, "batch": B, "ms_per_step": round(dt * 1e3, 3),
              "utterances_per_s": round(B / dt, 1), "gemm_dtype": prec})

    # ---- DABA selection: 60 pool triggers + 3000 hosts (trigger + poisoned host each)
    if not only or "daba_select" in only:
        torch.manual_seed(35)
        sel = D.DabaSelector(smallcnn(10, 896).to(dev), dev)
        r = np.random.default_rng(0)
        pool = [np.clip(r.normal(0, 4000, 16000), -32768, 32767).astype(np.int16) for _ in range(60)]
        hosts = [np.clip(r.normal(0, 4000, int(r.integers(9000, 16001))), -32768, 32767).astype(np.int16)
                 for _ in range(3000)]
        dt = timed(lambda: (sel.certainty(pool), sel.influence(pool[0], hosts)), max(3, args.steps // 4), warmup=1)
        emit({"workload": "daba_selection", "what": "Cer (60 pool triggers) + Inf (3000 hosts): overlay, librosa "
              "MFCC, 6060 per-utterance train-mode forwards, scores (host packing included)",
              "ms": round(dt * 1e3, 2), "forwards_per_s": round(6060 / dt, 1)})
        x = sel.clip_inputs(hosts[:2048] * 2)
        dtf = timed(lambda: sel.sel.log_probs(x), args.steps)
        emit({"workload": "daba_select_forward", "what": "per-utterance BN forward only, B=4096 (32x40)",
              "ms": round(dtf * 1e3, 3), "forwards_per_s": round(4096 / dtf, 1)})

    # ---- JingleBack style 5 board over the poisoned clips
    if not only or "styles" in only:
        waves, _ = synth.make_clips_torch(2048, 16000, 16000, 10, seed=6, device=dev)
        board = TR.get_boards()[5]
        for n in (256, 2048):
            w = waves[:n].contiguous()
            dt = timed(lambda: board.apply_device(w, 16000), args.steps)
            emit({"workload": f"style5_board:{n}", "what": "Gain(12) -> LadderFilter(HPF12, 1 kHz) -> Phaser()",
                  "clips": n, "ms": round(dt * 1e3, 3), "clips_per_s": round(n / dt, 1)})

    # ---- resample 16 kHz -> 44.1 kHz (prepare_dataset.py:60)
    if not only or "resample" in only:
        waves, _ = synth.make_clips_torch(2048, 16000, 16000, 10, seed=7, device=dev)
        dt = timed(lambda: F.resample(waves, 16000, 44100), args.steps)
        flops = 2048 * 44100 * 174 * 2
        emit({"workload": "resample_16k_44k1", "clips": 2048, "ms": round(dt * 1e3, 3),
              "clips_per_s": round(2048 / dt, 1), "tflops": round(flops / dt / 1e12, 2),
              "hbm_gbps": round(2048 * (16000 + 44100) * 4 / dt / 1e9, 1)})


if __name__ == "__main__":
    main()
