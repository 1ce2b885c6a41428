#!/usr/bin/env python3
"""Headline bench: poisoned+clean utterances/s through the full per-batch hot path.

Workload (BASELINE.json configs[1], the metric's own config): ultrasonic.py --
44.1 kHz x 1 s clips resident in HBM, 35 classes, per-GPU batch 512, fp32:
gather -> ultrasonic trigger add (10 % poisoned, target 2) -> STFT (n_fft 1103,
Bluestein) / mel / dB / DCT -> smallcnn forward+backward+CE -> [RCCL all-reduce]
-> Adam -> device counters.  One "step" = one such batch per GPU.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Rank 0 prints ONE JSON line (value = whole-job utterances/s, max time over ranks).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

FP32_MFMA_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: FP32 matrix 157.3 TF (spec; 155 measured)
BF16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: BF16 dense ~2.5 PF (no sparsity)
BF16_PHASES = ("conv2_fwd", "conv2_dgrad", "conv3_fwd", "conv3_dgrad")  # smallcnn GEMMs the bf16 modes move
SPLIT_TERMS = 6                 # f32split: six bf16 MFMA terms per fp32-accurate product
HBM_PEAK_GBPS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def algorithmic_work(phase, B, H0, W0, K, n_mels, T, C, L):
    """(amount, unit, bound) per launch of a libabd phase (DESIGN.md 'Roofline')."""
    H1, W1 = H0 - 1, W0 - 1
    W1p = W1 // 3
    H2, W2 = H1 - 1, W1p - 1
    H2p, W2p = H2 // 2 + 1, W2 // 2 + 1
    H3, W3 = H2p - 1, W2p - 1
    H3p, W3p = (H3 - 2) // 2 + 1, W3 // 2 + 1
    flat = 32 * H3p * W3p
    fl = {
        "conv2_fwd": 2.0 * B * H2 * W2 * 64 * 256,
        "conv2_wgrad": 2.0 * B * H2 * W2 * 64 * 256,
        "conv2_dgrad": 2.0 * B * H1 * W1p * 64 * 256,
        "conv3_fwd": 2.0 * B * H3 * W3 * 32 * 256,
        "conv3_wgrad": 2.0 * B * H3 * W3 * 32 * 256,
        "conv3_dgrad": 2.0 * B * H2p * W2p * 64 * 128,
        "fc1_fwd": 2.0 * B * 128 * flat,
        "fc1_wgrad": 2.0 * B * 128 * flat,
        "fc1_dgrad": 2.0 * B * 128 * flat,
    }
    if phase in fl:
        return fl[phase] / 1e12, "TFLOP/s", "mfma"
    by = {
        # wave read + mel-dB workspace write (trigger/tables amortised)
        "stft_mel": B * (4.0 * L + 4.0 * T * n_mels),
        "db_dct": B * (4.0 * T * n_mels + 4.0 * T * C),
        "bn2_bwd": B * H2 * W2 * 64 * 4.0 * 3,   # r2 (stats) + r2 read + dz2 write
        "bn2_pool": B * (H2 * W2 + H2p * W2p) * 64 * 4.0,
        "conv1_bwd_wgrad": B * (H0 * W0 + H1 * W1p * 64) * 4.0,
        "conv1_bn_pool": B * (H0 * W0 + H1 * W1p * 64) * 4.0,
    }
    if phase in by:
        return by[phase] / 1e9, "GB/s", "hbm"
    return None


def stft_flops(B, T, M=2304):
    """FFT arithmetic of one Bluestein STFT launch: two complex M-point FFTs (5 M log2 M) per pair of frames."""
    import math
    pairs = B * ((T + 1) // 2)
    return pairs * 2 * 5.0 * M * math.log2(M)


WORKLOADS = {
    "ultrasonic": "ultrasonic.py (BASELINE configs[1]): 44.1 kHz x 1 s clips resident in HBM, trigger add + HIP "
                  "STFT (n_fft 1103 Bluestein)/mel/dB/DCT -> (1,100,40) + smallcnn train step (fwd/bwd/CE/Adam) + "
                  "ASR/acc counters",
    "badnets": "badnets.py (BASELINE configs[0] shape on the GPU): 16 kHz MFCC (400/160) + BadNets patch + smallcnn step",
    "jingleback": "jingleback.py (BASELINE configs[2]): style-5 board clips resident, 16 kHz MFCC + smallcnn step",
    "daba": "daba.py (BASELINE configs[3]): librosa MFCC (2048/512, Slaney) 32x40 + smallcnn step",
    "flowmur": "flowmur.py (BASELINE configs[4]): SNR-30 trigger mix + MFCC (2048/512, 13) + smallcnn step",
}


def mfma_peak(phase, precision=None):
    """Dense MFMA peak of the dtype a phase's GEMM runs in (bf16 mode moves the conv fwd/dgrad GEMMs)."""
    prec = precision or _PRECISION[0]
    if phase in BF16_PHASES and prec == "bf16":
        return BF16_MFMA_PEAK_TFLOPS
    if phase in BF16_PHASES and prec == "f32split":   # fp32 FLOPs at the bf16 rate / six terms
        return BF16_MFMA_PEAK_TFLOPS / SPLIT_TERMS
    return FP32_MFMA_PEAK_TFLOPS


_PRECISION = ["f32split"]


def load_traffic(phase):
    """HBM bytes per launch from the committed rocprofv3 PMC pass (profiles/*traffic*.json), if any."""
    import glob
    for f in sorted(glob.glob(os.path.join(HERE, "profiles", "*traffic*.json")), reverse=True):
        try:
            d = json.load(open(f))
            if phase in d.get("bytes_per_launch", {}):
                return d["bytes_per_launch"][phase]
        except Exception:
            pass
    return None


def cpu_baseline(n, threads):
    """The float64 numpy oracle (port of the reference path) on a bounded sample, host cores."""
    import numpy as np
    from threadpoolctl import threadpool_limits
    from abd_amd import synth
    from abd_amd.pipeline import ultrasonic_trigger
    from oracle import mfcc as om, smallcnn as oc
    from tests.golden_inputs import make_state
    w, lab = synth.make_clips_np(n, 44100, 44100, 35, seed=123)
    trig = ultrasonic_trigger(60, "mid", False).astype(np.float64)
    r = np.random.Generator(np.random.PCG64(1))
    pois = r.random(n) < 0.1
    lab = np.where(pois, 2, lab)
    with threadpool_limits(limits=threads):
        t0 = time.perf_counter()
        ww = w.astype(np.float64)
        ww[pois] += trig[None]
        x = om.mfcc_model_input(ww, 44100, 40, 1103, 441)
        m = oc.SmallCNN(make_state(100, 40, 35, 3072, seed=5))
        m.train_step(x, lab, r.random((n, 3072)) < 0.6, r.random((n, 128)) < 0.5)
        dt = time.perf_counter() - t0
    return {"value": round(n / dt, 2), "unit": "utterances/s", "cores": threads, "kind": "port",
            "sample": f"{n} ultrasonic utterances (44.1 kHz x 1 s): trigger add + MFCC(1103/441) + one smallcnn "
                      f"train step (fwd/bwd/Adam), float64 numpy oracle, {dt:.1f} s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=512, help="per-GPU batch (configs[1]: bs=512)")
    ap.add_argument("--n-train", type=int, default=8192, help="resident training clips per GPU")
    ap.add_argument("--cpu-sample", type=int, default=192, help="utterances for the CPU baseline (0 = skip)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--profile-steps", type=int, default=3, help="untimed per-phase profiling steps after warmup")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL) on the node; gloo for 1-GPU rehearsal")
    ap.add_argument("--overlap", action="store_true", help="prefetch the next batch's features on a side stream")
    ap.add_argument("--attack", default="ultrasonic", help="workload: ultrasonic (headline, configs[1]), badnets, "
                    "jingleback, daba, flowmur")
    ap.add_argument("--gemm-precision", default="f32split", choices=("f32", "f32split", "bf16"),
                    help="conv GEMM precision (f32split, the default: fp32-accurate products as exact 3-way bf16 "
                         "splits on bf16 MFMA, parity-tested at the fp32 tolerance; f32: fp32 MFMA; "
                         "bf16: BASELINE configs[2])")
    args = ap.parse_args()
    _PRECISION[0] = args.gemm_precision

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()
    dev = torch.device("cuda", local % max(ndev, 1))  # rehearsal: several ranks may share one GPU
    torch.cuda.set_device(dev)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.dist_backend)

    import abd_amd
    from abd_amd import _lib as L
    from abd_amd import synth
    from abd_amd.models import smallcnn
    from abd_amd.pipeline import ResidentTrainer, attack_config, ultrasonic_trigger

    abd_amd.load_library()
    cfg = attack_config(args.attack)
    headline = args.attack == "ultrasonic" and args.gemm_precision in ("f32", "f32split")
    K = 35 if args.attack == "ultrasonic" else 10
    waves, labels = synth.make_clips_torch(args.n_train, cfg.sample_rate, cfg.length, K, seed=35 + rank, device=dev)
    if cfg.clean_label:  # FlowMur poisons target-class clips only: make sure there are some
        labels[: args.n_train // 4] = cfg.target_label
    trigger = None
    if args.attack == "ultrasonic":
        trigger = ultrasonic_trigger(60, "mid", False)
    elif args.attack == "flowmur":
        import numpy as np
        trigger = (0.05 * np.random.default_rng(1).standard_normal(8000)).astype(np.float32)
    torch.manual_seed(35)
    model = smallcnn(K, cfg.linear_features).to(dev)
    opt = torch.optim.Adam(model.parameters(), lr=1e-4)
    tr = ResidentTrainer(cfg, waves, labels, model, opt, args.batch, trigger=trigger, seed=35, rank=rank,
                         world=world, overlap_features=args.overlap, gemm_precision=args.gemm_precision)

    # warmup (untimed), then a few more untimed steps with every libabd phase bracketed to
    # find the dominant kernel in steady state
    for _ in range(args.warmup):
        tr.step()
    torch.cuda.synchronize()
    with L.PhaseProfiler(L.PHASES, max_records=64 * args.profile_steps) as wprof:
        for _ in range(args.profile_steps):
            tr.step()
        torch.cuda.synchronize()
    phases_ms = {k: round(v[0] / max(v[1], 1), 4) for k, v in wprof.result.items()}
    dominant = max(wprof.result, key=lambda k: wprof.result[k][0]) if wprof.result else "conv2_dgrad"

    prof = L.PhaseProfiler([dominant], max_records=args.steps + 4)
    prof.__enter__()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        tr.step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    prof.__exit__(None, None, None)
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    metrics = tr.read_metrics()

    if rank == 0:
        n_utt = args.batch * world * args.steps
        ms, cnt = prof.result.get(dominant, (0.0, 0))
        avg_s = ms / max(cnt, 1) / 1e3
        T, C, L_ = tr.T, cfg.n_mfcc, cfg.length
        work = algorithmic_work(dominant, args.batch, T, C, K, 128, T, C, L_)
        roof = None
        if work is not None and avg_s > 0:
            amount, unit, bound = work
            achieved = amount / avg_s
            peak = mfma_peak(dominant) if bound == "mfma" else HBM_PEAK_GBPS
            roof = {"kernel": dominant, "bound": bound, "achieved": round(achieved, 3), "peak": peak, "unit": unit,
                    "frac": round(achieved / peak, 4), "traffic": load_traffic(dominant) if headline else None,
                    "avg_launch_ms": round(avg_s * 1e3, 4), "launches": cnt}
        # every phase with an algorithmic work model, from the untimed per-phase profiling steps
        per_kernel = {}
        for ph, (pms, pcnt) in wprof.result.items():
            wk = algorithmic_work(ph, args.batch, T, C, K, 128, T, C, L_)
            if wk is None or pcnt == 0 or pms <= 0:
                continue
            amt, unit, bnd = wk
            ach = amt / (pms / pcnt / 1e3)
            pk = mfma_peak(ph) if bnd == "mfma" else HBM_PEAK_GBPS
            per_kernel[ph] = {"bound": bnd, "achieved": round(ach, 2), "unit": unit, "frac": round(ach / pk, 4),
                              "ms": round(pms / pcnt, 4), "traffic": load_traffic(ph) if headline else None}
        if roof is not None and dominant == "stft_mel" and args.attack == "ultrasonic":
            # the STFT moves few bytes per FLOP: its real limit is VALU issue (FFT butterflies),
            # reported beside the HBM fraction the metric asks for
            roof["note"] = ("HBM-bound by the survey's byte model but VALU-limited in practice: "
                            f"{stft_flops(args.batch, T) / avg_s / 1e12:.1f} TFLOP/s of FFT arithmetic "
                            f"(fp32 vector peak {FP32_MFMA_PEAK_TFLOPS})")
        cpu = None
        if world == 1 and not args.no_cpu and args.cpu_sample > 0 and args.attack == "ultrasonic":
            threads = min(16, len(os.sched_getaffinity(0)))
            cpu = cpu_baseline(args.cpu_sample, threads)
        line = {
            "metric": "poisoned+clean utterances/sec/GPU; ASR & clean-acc parity vs reference",
            "value": round(n_utt / dt, 1),
            "unit": "utterances/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": {"f32": "f32", "f32split": "f32 (conv GEMMs as exact 3-way bf16 splits, 6 MFMA terms, fp32 accumulate)"}.get(
                args.gemm_precision, "bf16 conv GEMMs (fp32 accumulate), fp32 elsewhere"),
            "data": "synthetic",
            "config": {"workload": WORKLOADS[args.attack], "attack": args.attack, "num_classes": K,
                       "gemm_precision": args.gemm_precision, "per_gpu_batch": args.batch,
                       "global_batch": args.batch * world, "poisoning_rate": cfg.poisoning_rate,
                       "resident_clips_per_gpu": args.n_train, "parallelism": f"dp{world}"},
            "roofline": roof,
            "cpu_baseline": cpu,
            "phases_ms_per_launch": phases_ms,
            "roofline_by_kernel": per_kernel,
            "train_metrics": {k: round(v, 4) if isinstance(v, float) else v for k, v in metrics.items()},
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
