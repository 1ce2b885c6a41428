#!/usr/bin/env python3
"""Headline bench: poisoned+clean utterances/s through the full per-batch hot path.

Workload (BASELINE.json configs[1], the metric's own config): ultrasonic.py --
44.1 kHz x 1 s clips resident in HBM, 35 classes, per-GPU batch 512, fp32:
gather -> ultrasonic trigger add (10 % poisoned, target 2) -> STFT (n_fft 1103,
Bluestein) / mel / dB / DCT -> smallcnn forward+backward+CE -> [RCCL all-reduce]
-> Adam -> device counters.  One "step" = one such batch per GPU.

    python bench.py [--gpus N --steps K --warmup W]       # N > 1: spawns the N ranks itself
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...   # WORLD_SIZE must equal N

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
# smallcnn GEMMs the bf16 / f32split modes run on bf16 MFMA (the weight gradients through
# conv_wgrad_trp_kernel: six split terms in f32split, one bf16 term in bf16)
BF16_PHASES = ("conv2_fwd", "conv2_dgrad", "conv3_fwd", "conv3_dgrad", "conv2_wgrad", "conv3_wgrad")
SPLIT_TERMS = 6                 # f32split: six bf16 MFMA terms per fp32-accurate product
HBM_PEAK_GBPS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
FP32_VECTOR_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: Peak FP32 (vector) 157.3 TF
VALU_CLOCK_GHZ = 2.4  # peak engine clock: one wave64 VALU issue per CU-cycle (non-packed)


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
        # fused fc head (fc_head.inc), priced on its dense GEMMs (fp32 MFMA): head_fwd = fc1 forward
        # (+ pool3 / BN3 / dropout1), head_mid = the per-row head (fc2 forward and its data
        # gradient, + loss), head_dgrad = fc1 data gradient (+ dropout1' and BN3's sums),
        # head_bwd = fc1 weight gradient (+ fc2 gradients and BN3's backward apply)
        "head_fwd": 2.0 * B * 128 * flat,
        "head_mid": 2.0 * 2.0 * B * 128 * K,
        "head_dgrad": 2.0 * B * 128 * flat,
        "head_bwd": 2.0 * B * 128 * flat,
    }
    if phase in fl:
        return fl[phase] / 1e12, "TFLOP/s", "mfma"
    by = {
        # wave read + mel-dB workspace write (trigger/tables amortised)
        "stft_mel": B * (4.0 * L + 4.0 * T * n_mels),
        "db_dct": B * (4.0 * T * n_mels + 4.0 * T * C),
        # bn_bwd_apply_kernel: r2 read + pooled gradient dp2 read + dz2 write (the statistics pass
        # over r2 left the step in round 2: BN2's sums are derived from conv3's gradients)
        "bn2_bwd": B * (2.0 * H2 * W2 + H2p * W2p) * 64 * 4.0,
        "bn2_pool": B * (H2 * W2 + H2p * W2p) * 64 * 4.0,        # r2 read + p2 write
        "conv1_bwd_wgrad": B * (H0 * W0 + H1 * W1p * 64) * 4.0,   # x read + dp1 read
        "conv1_bn_pool": B * (H0 * W0 + H1 * W1p * 64) * 4.0,
        "conv1_stats": B * (H0 * W0 + H1 * W1p * 64) * 4.0,       # x read + pool1-selected m write (fold)
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


_TRAFFIC = []


def traffic_file():
    """The committed rocprofv3 FETCH/WRITE measurement (profiles/*traffic*.json, scripts/traffic_json.py)
    taken on THESE libabd sources (its csrc_sha1 equals theirs), newest first; None if there is none --
    an older measurement of different kernels is never used."""
    if not _TRAFFIC:
        import glob
        sys.path.insert(0, os.path.join(HERE, "scripts"))
        from traffic_json import csrc_sha1
        sha, found = csrc_sha1(HERE), None
        for f in sorted(glob.glob(os.path.join(HERE, "profiles", "*traffic*.json")), key=os.path.getmtime,
                        reverse=True):
            try:
                d = json.load(open(f))
            except Exception:
                continue
            if d.get("csrc_sha1") == sha:
                found = (os.path.relpath(f, HERE), d)
                break
        _TRAFFIC.append(found)
    return _TRAFFIC[0]


def load_valu_insts(phase):
    """(VALU wave-instructions per launch, source file) for a phase from the same-source traffic file's
    SQ_INSTS_VALU pass, else (None, None)."""
    tf = traffic_file()
    if tf is None or phase not in tf[1].get("valu_insts_per_launch", {}):
        return None, None
    return tf[1]["valu_insts_per_launch"][phase], tf[0]


def load_traffic(phase):
    """(HBM bytes per launch, source file) for a phase from the same-source traffic file, else (None, None)."""
    tf = traffic_file()
    if tf is None or phase not in tf[1].get("bytes_per_launch", {}):
        return None, None
    return tf[1]["bytes_per_launch"][phase], tf[0]


def cpu_threads():
    """Host threads for the CPU baseline: this process's CPU affinity, capped by OMP_NUM_THREADS
    (the GPU box exports 16, its CPU share; its affinity mask shows the whole machine)."""
    n = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(n, int(omp))) if omp and omp.isdigit() else n


def cpu_baseline(batch, threads, n_train=4096, n_test=1024, warmup_steps=5):
    """The reference CPU path on the bench's workload (5 warmup steps, one timed
    epoch, clean accuracy / ASR after it), as a bounded sample -- 4,096 of BASELINE's 20,480 training
    clips, so the default bench finishes in minutes (the task's 10-30 s CPU budget) -- on the box's
    CPU share (OMP_NUM_THREADS, 16; `affinity_cpus` reports sched_getaffinity, the whole host): torch-fp32
    restatement (oracle/torch_ref.py: torch.stft MFCC with torchaudio's semantics + nn smallcnn of the
    reference structure + torch Adam), ultrasonic K = 35, 10 % of the training clips poisoned.  After
    `warmup_steps` untimed steps, ONE full epoch over n_train clips at the bench batch is timed (per
    batch, as in the GPU step: trigger add on the poisoned rows -> MFCC -> forward / CE / backward /
    Adam -> counters); then test() on n_test clean clips and on the backdoor test set (the non-target
    test clips with the trigger, labels 2) gives clean accuracy and ASR after that epoch."""
    import numpy as np
    import torch
    from oracle import torch_ref
    sys.path.insert(0, os.path.join(HERE, "tests"))
    from golden_inputs import ultrasonic_trigger_f32
    from abd_amd import synth
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        t_prep = time.perf_counter()
        waves, labels = synth.make_clips_torch(n_train + n_test, 44100, 44100, 35, seed=123, device="cpu")
        trig = torch.from_numpy(ultrasonic_trigger_f32()[0])
        feat = torch_ref.MfccCPU(44100, 40, 1103, 441)
        torch.manual_seed(5)
        model = torch_ref.SmallCNN(35, 3072).train()
        opt = torch.optim.Adam(model.parameters(), lr=1e-4)
        g = torch.Generator().manual_seed(1)
        tr_w, tr_y = waves[:n_train], labels[:n_train]
        pois = torch.zeros(n_train, dtype=torch.bool)
        pois[torch.randperm(n_train, generator=g)[: n_train // 10]] = True        # ultrasonic.py:70-71
        y_eff = torch.where(pois, torch.full_like(tr_y, 2), tr_y)                  # :77

        def step(rows):
            x = tr_w[rows] + pois[rows, None].float() * trig[None]                 # ultrasonic.py:75
            return torch_ref.train_step(model, opt, feat(x), y_eff[rows], pois[rows].long())
        warm = torch.randperm(n_train, generator=g)
        for k in range(warmup_steps):   # wraps around a table smaller than warmup_steps x batch
            step(warm[(torch.arange(batch) + k * batch) % n_train])
        prep_s = time.perf_counter() - t_prep
        perm = torch.randperm(n_train, generator=g)
        loss, correct, ptot, phit, nb = 0.0, 0, 0, 0, 0
        t0 = time.perf_counter()
        for s0 in range(0, n_train, batch):
            l_, c_, p_, h_ = step(perm[s0:s0 + batch])
            loss, correct, ptot, phit, nb = loss + l_, correct + c_, ptot + p_, phit + h_, nb + 1
        dt = time.perf_counter() - t0
        model.eval()
        te_w, te_y = waves[n_train:], labels[n_train:]
        with torch.no_grad():
            pred = torch.cat([model(feat(te_w[s:s + 256])).argmax(1) for s in range(0, n_test, 256)])
            bd = te_y != 2                                                       # ultrasonic.py:90-102
            bw = te_w[bd] + trig[None]
            bpred = torch.cat([model(feat(bw[s:s + 256])).argmax(1) for s in range(0, bw.shape[0], 256)])
        epoch = {"train_loss": round(loss / nb, 4), "train_acc": round(100.0 * correct / n_train, 3),
                 "train_asr": round(100.0 * phit / max(ptot, 1), 3),
                 "clean_acc": round(100.0 * float((pred == te_y).float().mean()), 3),
                 "asr": round(100.0 * float((bpred == 2).float().mean()), 3)}
    finally:
        torch.set_num_threads(prev)
    return {"value": round(n_train / dt, 2), "unit": "utterances/s", "cores": threads,
            "affinity_cpus": len(os.sched_getaffinity(0)), "kind": "port",
            "sample": f"one epoch of {n_train} clips at batch {batch} ({nb} steps, {dt:.1f} s) after {warmup_steps} "
                      f"warmup steps: ultrasonic clips (44.1 kHz x 1 s, 10 % poisoned), trigger add + torch.stft "
                      f"MFCC(1103/441) + smallcnn fwd/bwd/Adam in torch fp32 on {threads} host threads "
                      f"(oracle/torch_ref.py, the reference CPU path restated); then test() on {n_test} clean clips "
                      f"and {int(bd.sum())} backdoor clips",
            "epoch_s": round(dt, 3), "setup_s": round(prep_s, 3), "after_epoch": epoch}


def dropin_bench(cfg, waves, K, batch, nbatch, dev, precision):
    """The unchanged attack scripts' loop (utils/training_tools.py:52-85 train(), badnets.py:146-160):
    the drop-in ``train()`` over a DataLoader of precomputed (1, T, C) MFCC, per-batch H2D included --
    against the same device step without the Python loop (what ResidentTrainer runs per batch after
    its feature stage).  Four timings over `nbatch` batches of `batch` rows, each after a warmup:
    cnn_step (training.train_step on device-resident batches: the resident CNN phases), dropin_device
    (train() over already-resident batches: the drop-in's Python + custom-op dispatch around the same
    step), dropin_loader (train() over the scripts' DataLoader(BDDataset, shuffle=True): the resident
    fast path, resident.py), dropin_host_loader (the same loader forced through per-batch host
    collation + pageable H2D, as the reference iterates it), loader_only."""
    import torch
    from torch.utils.data._utils.collate import default_collate
    from abd_amd import features as F, training as T, _lib as L
    from abd_amd.models import smallcnn
    from abd_amd.resident import BDDataset   # prepare_dataset.py:13-33 (the drop-in's class)

    mcfg = cfg.mfcc()
    n = batch * nbatch
    rows = torch.arange(n, dtype=torch.int32, device=dev) % waves.shape[0]
    xs = torch.cat([F.mfcc_batch(waves, mcfg, rows=rows[s:s + batch]) for s in range(0, n, batch)])
    g = torch.Generator().manual_seed(3)
    y = torch.randint(0, K, (n,), generator=g)
    ind = (torch.rand(n, generator=g) < cfg.poisoning_rate).long()
    y[ind == 1] = cfg.target_label
    x_cpu = xs.cpu()
    dev_batches = [{"mfcc": xs[s:s + batch], "label": y[s:s + batch].to(dev), "poison_indicator": ind[s:s + batch].to(dev)}
                   for s in range(0, n, batch)]
    loader = torch.utils.data.DataLoader(BDDataset(x_cpu, y, ind), batch_size=batch, shuffle=True)
    host_loader = torch.utils.data.DataLoader(BDDataset(x_cpu, y, ind), batch_size=batch, shuffle=True,
                                              collate_fn=lambda b: default_collate(b))
    crit = torch.nn.CrossEntropyLoss()

    def fresh():
        torch.manual_seed(35)
        m = smallcnn(K, cfg.linear_features).to(dev).set_gemm_precision(precision)
        return m, torch.optim.Adam(m.parameters(), lr=1e-4)

    def timed(fn):
        fn()                      # warmup pass (binds the engine, allocates workspaces)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3 / nbatch

    m0, o0 = fresh()
    m0.train()
    T.train(m0, dev_batches[:1], dev, o0, crit)
    adam = T.AdamBinding(m0, o0)
    met = torch.zeros(L.METRICS_WORDS, dtype=torch.int64, device=dev)
    res = {"cnn_step_ms": timed(lambda: [T.train_step(m0, b["mfcc"], b["label"], b["poison_indicator"], adam, met)
                                         for b in dev_batches])}
    m1, o1 = fresh()
    res["dropin_device_ms"] = timed(lambda: T.train(m1, dev_batches, dev, o1, crit))
    m2, o2 = fresh()
    res["dropin_loader_ms"] = timed(lambda: T.train(m2, loader, dev, o2, crit))
    m3, o3 = fresh()
    res["dropin_host_loader_ms"] = timed(lambda: T.train(m3, host_loader, dev, o3, crit))
    t0 = time.perf_counter()
    for _ in host_loader:
        pass
    res["loader_only_ms"] = (time.perf_counter() - t0) * 1e3 / nbatch
    res = {k: round(v, 4) for k, v in res.items()}
    res["dropin_device_vs_cnn_step"] = round(res["dropin_device_ms"] / res["cnn_step_ms"], 4)
    res["dropin_loader_vs_device"] = round(res["dropin_loader_ms"] / res["dropin_device_ms"], 4)
    res["batches"], res["batch"], res["gemm_precision"] = nbatch, batch, precision
    res["note"] = ("train() over a DataLoader of precomputed MFCC (the reference scripts' loop, badnets.py:146-160); "
                   "dropin_device excludes the loader (batches already in HBM); dropin_loader iterates the scripts' "
                   "DataLoader(BDDataset, shuffle=True) through the HBM-resident fast path (same batches and RNG "
                   "consumption, rows gathered on the device); dropin_host_loader forces the reference's per-batch "
                   "host collation and pageable-memory H2D of each batch")
    return res


FEATURE_PHASES = ("stft_mel", "db_dct")


def feature_bytes(L, T, C):
    """SURVEY §8(d) algorithmic bytes per utterance of the feature stage: wave read + MFCC write."""
    return 4.0 * L + 4.0 * T * C


def train_flops(H0, W0, K):
    """3 F_fwd - F_conv1 per utterance (conv + linear, 2 FLOP per MAC)."""
    H1, W1 = H0 - 1, W0 - 1
    W1p = W1 // 3
    H2, W2 = H1 - 1, W1p - 1
    H2p, W2p = H2 // 2 + 1, W2 // 2 + 1
    H3, W3 = H2p - 1, W2p - 1
    H3p, W3p = (H3 - 2) // 2 + 1, W3 // 2 + 1
    flat = 32 * H3p * W3p
    c1 = 2.0 * H1 * W1 * 64 * 4
    fwd = c1 + 2.0 * H2 * W2 * 64 * 256 + 2.0 * H3 * W3 * 32 * 256 + 2.0 * flat * 128 + 2.0 * 128 * K
    return 3.0 * fwd - c1


def rank_envs(n, port, base=None):
    """Per-rank environments of an N-rank launch on this node (what torch.distributed.run exports)."""
    base = dict(os.environ if base is None else base)
    out = []
    for r in range(n):
        e = dict(base)
        e.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(n), "LOCAL_WORLD_SIZE": str(n),
                  "GROUP_RANK": "0", "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
        out.append(e)
    return out


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _relay(stream, rank):
    """Forward a rank's stdout: rank 0's JSON line(s) to this process's stdout, every other line
    (collective libraries print connection banners to stdout) to stderr."""
    for raw in iter(stream.readline, b""):
        line = raw.decode(errors="replace")
        out = sys.stdout if rank == 0 and line.lstrip().startswith("{") else sys.stderr
        out.write(line)
        out.flush()
    stream.close()


def spawn_ranks(n, cmd, poll_s=0.2):
    """`bench.py --gpus N` without a launcher: start N fresh child processes (one per GPU, rank r on
    cuda:r) running `cmd` with the rendezvous environment, wait for all of them and return the first
    non-zero exit status (0 if every rank succeeded).  Called BEFORE anything touches the GPU -- this
    process never imports torch -- so each child initialises HIP itself.  Rank 0's JSON line is
    relayed to stdout, everything else the ranks print goes to stderr; if one rank fails the others
    are terminated instead of being left waiting in a collective."""
    import signal
    import subprocess
    import threading
    procs = [subprocess.Popen(cmd, env=e, stdout=subprocess.PIPE) for e in rank_envs(n, free_port())]
    relays = [threading.Thread(target=_relay, args=(p.stdout, r), daemon=True) for r, p in enumerate(procs)]
    for t in relays:
        t.start()
    stopped = []

    def stop(*_):
        # SIGTERM first; SIGKILL after a grace period (a rank may inherit SIGTERM ignored)
        if not stopped:
            stopped.append(time.time())
        for p in procs:
            if p.poll() is None:
                p.terminate() if time.time() - stopped[0] < 5.0 else p.kill()
    old = signal.signal(signal.SIGTERM, lambda *a: (stop(), sys.exit(143)))
    try:
        status = 0
        while [p.poll() for p in procs].count(None):   # poll every rank (any() would stop at the first)
            bad = [p.returncode for p in procs if p.returncode not in (None, 0)]
            if bad:
                status = status or bad[0]
                stop()
            time.sleep(poll_s)
        for p in procs:
            p.wait()
            if p.returncode != 0 and status == 0:
                status = p.returncode
        for t in relays:
            t.join(timeout=10.0)
        return status if status >= 0 else 128 - status
    finally:
        signal.signal(signal.SIGTERM, old)


def resolve_world(gpus, environ=None):
    """(world, spawn): the launch `--gpus N` asks for.  Under a launcher (WORLD_SIZE set) the launcher's
    world must equal N; without one, N > 1 means this process spawns the N ranks itself."""
    environ = os.environ if environ is None else environ
    if gpus < 1:
        raise SystemExit(f"bench.py: --gpus must be >= 1 (got {gpus})")
    ws = environ.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != gpus:
            raise SystemExit(f"bench.py: WORLD_SIZE={ws} from the launcher disagrees with --gpus {gpus}")
        return gpus, False
    return gpus, gpus > 1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=512, help="per-GPU batch (configs[1]: bs=512)")
    ap.add_argument("--n-train", type=int, default=8192, help="resident training clips per GPU (the table is "
                    "replicated on every rank and holds n_train x world clips, so an epoch has the same number "
                    "of steps at every N)")
    ap.add_argument("--cpu-train", type=int, default=4096, help="CPU-baseline epoch size in clips (0 = skip)")
    ap.add_argument("--dropin-batches", type=int, default=16, help="batches of the drop-in train() measurement "
                    "(0 = skip; rank 0 at N = 1 only)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--profile-steps", type=int, default=3, help="untimed per-phase profiling steps after warmup")
    ap.add_argument("--profile-every", type=int, default=4,
                    help="timed steps: HIP-event brackets on every n-th launch of the dominant kernel(s) only "
                         "(each bracket serialises the stream, ~4-5 us of idle GPU per event)")
    ap.add_argument("--windows", type=int, default=5, help="equal windows of the timed steps (median reported)")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL) on the node; gloo for 1-GPU rehearsal")
    ap.add_argument("--sync-bn", action="store_true", help="BatchNorm statistics over the global batch")
    ap.add_argument("--attack", default="ultrasonic", help="workload: ultrasonic (headline, configs[1]), badnets, "
                    "jingleback, daba, flowmur")
    ap.add_argument("--gemm-precision", default="f32split", choices=("f32", "f32split", "bf16"),
                    help="conv GEMM precision (f32split, the default: fp32-accurate products as exact 3-way bf16 "
                         "splits on bf16 MFMA, parity-tested at the fp32 tolerance; f32: fp32 MFMA; "
                         "bf16: BASELINE configs[2])")
    args = ap.parse_args()
    _PRECISION[0] = args.gemm_precision
    world, spawn = resolve_world(args.gpus)
    if spawn:   # no launcher: this process only starts the ranks (it never touches the GPU)
        sys.exit(spawn_ranks(world, [sys.executable, os.path.abspath(__file__)] + sys.argv[1:]))

    import torch
    import torch.distributed as dist

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
    n_clips = args.n_train * world
    waves, labels = synth.make_clips_torch(n_clips, cfg.sample_rate, cfg.length, K, seed=35, device=dev)
    if cfg.clean_label:  # FlowMur poisons target-class clips only: make sure there are some
        labels[: n_clips // 4] = cfg.target_label
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
                         world=world, gemm_precision=args.gemm_precision, sync_bn=args.sync_bn)

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
    # the feature stage is measured as a unit (SURVEY §8d bytes: wave in, MFCC out)
    live = list(FEATURE_PHASES) if dominant in FEATURE_PHASES else [dominant]

    # timed region: exactly `steps` steps between barrier + synchronize; HIP events bracket the
    # dominant kernel(s) on their launch stream, plus one event per window boundary
    prof = L.PhaseProfiler(live, max_records=len(live) * args.steps + 8, every=max(1, args.profile_every))
    nwin = max(1, min(args.windows, args.steps))
    bounds = [round(i * args.steps / nwin) for i in range(nwin + 1)]
    wev = [torch.cuda.Event(enable_timing=True) for _ in bounds]
    prof.__enter__()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    wev[0].record()
    bi = 1
    for k in range(args.steps):
        prof.step()   # brackets sample whole steps: every launch of the live phases in every n-th step
        tr.step()
        if bi < len(bounds) and k + 1 == bounds[bi]:
            wev[bi].record()
            bi += 1
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    prof.__exit__(None, None, None)
    win_ms = [wev[i].elapsed_time(wev[i + 1]) / max(bounds[i + 1] - bounds[i], 1) for i in range(nwin)]
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    metrics = tr.read_metrics()

    if rank == 0:
        import statistics
        n_utt = args.batch * world * args.steps
        T, C, L_ = tr.T, cfg.n_mfcc, cfg.length
        roof = None
        ms_live = {ph: prof.result.get(ph, (0.0, 0)) for ph in live}
        cnt = min(c for _, c in ms_live.values()) if ms_live else 0
        avg_s = sum(ms / max(c, 1) for ms, c in ms_live.values()) / 1e3
        if cnt > 0 and avg_s > 0:
            if dominant in FEATURE_PHASES:
                amount = args.batch * feature_bytes(L_, T, C) / 1e9
                unit, bound, peak = "GB/s", "hbm", HBM_PEAK_GBPS
                traffic, tsrc = None, None
                if headline:
                    tb = [load_traffic(ph) for ph in live]
                    if all(v is not None for v, _ in tb):
                        traffic, tsrc = sum(v for v, _ in tb), tb[0][1]
            else:
                amount, unit, bound = algorithmic_work(dominant, args.batch, T, C, K, 128, T, C, L_)
                peak = mfma_peak(dominant) if bound == "mfma" else HBM_PEAK_GBPS
                traffic, tsrc = load_traffic(dominant) if headline else (None, None)
            achieved = amount / avg_s
            roof = {"kernel": "+".join(live), "bound": bound, "achieved": round(achieved, 3), "peak": peak,
                    "unit": unit, "frac": round(achieved / peak, 4), "traffic": traffic, "traffic_source": tsrc,
                    "algorithmic_bytes": round(amount * 1e9) if unit == "GB/s" else None,
                    "avg_launch_ms": round(avg_s * 1e3, 4), "launches": cnt,
                    "sampled_every": max(1, args.profile_every),
                    "sampling": "per step (every launch of the live phases in steps 0, n, 2n, ...)",
                    "launches_per_step": {ph: round(wprof.result.get(ph, (0, 0))[1] / max(args.profile_steps, 1), 3)
                                          for ph in live},
                    "formula": ("B*(4L + 4*T*C) / (avg stft_mel + avg db_dct) [SURVEY 8d feature bytes]"
                                if dominant in FEATURE_PHASES else "per-launch algorithmic FLOP / avg launch")}
            if dominant == "stft_mel" and args.attack == "ultrasonic":
                st_ms, st_c = ms_live["stft_mel"]
                roof["note"] = ("HBM-bound by the survey's byte model but VALU-limited in practice: "
                                f"{stft_flops(args.batch, T) / (st_ms / st_c / 1e3) / 1e12:.1f} TFLOP/s of FFT "
                                f"arithmetic in stft_mel (fp32 vector peak {FP32_MFMA_PEAK_TFLOPS})")
        # step-level roofline: ideal time per utterance = feature bytes / HBM + train FLOPs / fp32 peak
        H0, W0 = T, C
        t_ideal = args.batch * (feature_bytes(L_, T, C) / (HBM_PEAK_GBPS * 1e9)
                                + train_flops(H0, W0, K) / (FP32_MFMA_PEAK_TFLOPS * 1e12))
        step_s = dt / args.steps
        step_roof = {"t_ideal_ms": round(t_ideal * 1e3, 4), "t_step_ms": round(step_s * 1e3, 4),
                     "frac": round(t_ideal / step_s, 4), "feature_bytes_per_utt": feature_bytes(L_, T, C),
                     "train_flops_per_utt": train_flops(H0, W0, K),
                     "peaks": f"HBM {HBM_PEAK_GBPS} GB/s, fp32 MFMA {FP32_MFMA_PEAK_TFLOPS} TFLOP/s"}
        # every phase with an algorithmic work model, from the untimed per-phase profiling steps
        per_kernel = {}
        for ph, (pms, pcnt) in wprof.result.items():
            wk = algorithmic_work(ph, args.batch, T, C, K, 128, T, C, L_)
            if wk is None or pcnt == 0 or pms <= 0:
                continue
            amt, unit, bnd = wk
            ach = amt / (pms / pcnt / 1e3)
            pk = mfma_peak(ph) if bnd == "mfma" else HBM_PEAK_GBPS
            tb, tsrc = load_traffic(ph) if headline else (None, None)
            per_kernel[ph] = {"bound": bnd, "achieved": round(ach, 2), "unit": unit, "peak": pk, "frac": round(ach / pk, 4),
                              "ms": round(pms / pcnt, 4), "traffic": tb, "traffic_source": tsrc}
            vi, _ = load_valu_insts(ph) if headline else (None, None)
            if vi:  # VALU issue rate against one wave64 instruction per CU-cycle (same-source SQ pass)
                ncu = torch.cuda.get_device_properties(dev).multi_processor_count
                per_kernel[ph]["valu_issue_frac"] = round(vi / (pms / pcnt / 1e3) / (ncu * VALU_CLOCK_GHZ * 1e9), 4)
            if ph == "stft_mel" and cfg.n_fft == 1103:
                # the limiter the byte model misses: the Bluestein FFTs' arithmetic
                # (5 M log2 M per complex M-point FFT, two per frame pair) against the fp32 VECTOR
                # peak (MI355X_MICROARCH.md: 157.3 TF, 256 CUs x 4 SIMD-32 x FMA at 2.4 GHz)
                tf = stft_flops(args.batch, T) / (pms / pcnt / 1e3) / 1e12
                per_kernel["stft_mel_valu"] = {"bound": "valu", "achieved": round(tf, 2), "unit": "TFLOP/s",
                                               "peak": FP32_VECTOR_PEAK_TFLOPS,
                                               "frac": round(tf / FP32_VECTOR_PEAK_TFLOPS, 4),
                                               "ms": round(pms / pcnt, 4),
                                               "formula": "B * ceil(T/2) pairs * 2 FFTs * 5 M log2 M, M = 2304"}
                # and against the VALU issue limit: one wave64 VALU instruction per CU-cycle without
                # packed FP32 (4 SIMDs x 16 lanes; MI355X_MICROARCH.md), instructions counted by the
                # same-source SQ_INSTS_VALU pass
                vi, vsrc = load_valu_insts("stft_mel") if headline else (None, None)
                if vi:
                    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
                    gi = vi / (pms / pcnt / 1e3) / 1e9
                    pk = ncu * VALU_CLOCK_GHZ
                    per_kernel["stft_mel_issue"] = {"bound": "valu_issue", "achieved": round(gi, 1),
                                                    "unit": "G wave-instr/s", "peak": round(pk, 1),
                                                    "frac": round(gi / pk, 4), "ms": round(pms / pcnt, 4),
                                                    "valu_insts_per_launch": vi, "source": vsrc,
                                                    "formula": "SQ_INSTS_VALU per launch / launch time vs CUs x 2.4 GHz"}
        cpu = None
        if world == 1 and not args.no_cpu and args.cpu_train > 0 and args.attack == "ultrasonic":
            cpu = cpu_baseline(args.batch, cpu_threads(), n_train=args.cpu_train)
        dropin = None
        if world == 1 and args.dropin_batches > 0:
            dropin = dropin_bench(cfg, tr.waves, K, args.batch, args.dropin_batches, dev, args.gemm_precision)
            cnn = sum(v[0] for k, v in wprof.result.items() if k not in FEATURE_PHASES) / max(args.profile_steps, 1)
            dropin["resident_cnn_phase_ms_per_step"] = round(cnn, 4)
        value = n_utt / dt
        line = {
            "metric": "poisoned+clean utterances/sec/GPU; ASR & clean-acc parity vs reference",
            "value": round(value, 1),
            "unit": "utterances/s",
            "value_semantics": "whole-job utterances/s over all ranks (per-GPU figure in value_per_gpu)",
            "value_per_gpu": round(value / world, 1),
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 4),
            "ms_per_step_window_median": round(statistics.median(win_ms), 4),
            "ms_per_step_windows": [round(v, 4) for v in win_ms],
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": {"f32": "f32", "f32split": "f32 (conv GEMMs as exact 3-way bf16 splits, 6 MFMA terms, fp32 accumulate)"}.get(
                args.gemm_precision, "bf16 conv GEMMs (fp32 accumulate), fp32 elsewhere"),
            "data": "synthetic",
            "config": {"workload": WORKLOADS[args.attack], "attack": args.attack, "num_classes": K,
                       "gemm_precision": args.gemm_precision, "per_gpu_batch": args.batch,
                       "global_batch": args.batch * world, "poisoning_rate": cfg.poisoning_rate,
                       "resident_clips": n_clips, "sync_bn": bool(args.sync_bn), "parallelism": f"dp{world}"},
            "roofline": roof,
            "step_roofline": step_roof,
            "cpu_baseline": cpu,
            "dropin": dropin,
            "phases_ms_per_launch": phases_ms,
            "roofline_by_kernel": per_kernel,
            "train_metrics": {k: round(v, 4) if isinstance(v, float) else v for k, v in metrics.items()},
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
