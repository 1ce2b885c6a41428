#!/usr/bin/env python3
"""Where does the side-stream gradient all-reduce of a data-parallel step run?

Runs ResidentTrainer steps at the bench's workload (ultrasonic, B = 512, f32split) with
collectives=True on a world-1 process group, so the step takes the data-parallel path:
abd_train_args.fc_grads_event recorded mid-backward, OverlappedGradAllReduce.launch_fc issuing
the fc-tail all-reduce on a side stream that waits on that event, finish() joining before Adam.
Run under ``rocprofv3 --kernel-trace`` and read the trace with ``--report DIR``.

  --mode rccl       backend "nccl" (RCCL), world size 1
  --mode surrogate  the same plumbing, but the side stream runs a stand-in kernel in place of the
                    collective (an elementwise pass over the 1.58 MB fc tail, the bytes a ring
                    all-reduce moves per rank per direction): where a side-stream kernel enqueued
                    at fc_grads_event actually starts relative to the persistent conv kernels.

    rocprofv3 --kernel-trace -d gpurun_out/ov -o ov -f csv -- python3 scripts/overlap_trace.py --mode rccl
    python3 scripts/overlap_trace.py --report gpurun_out/ov
"""
import argparse
import csv
import glob
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

WATCH = (("conv2 dgrad", "conv_ws_spec_kernel<0, 2"), ("conv2 wgrad", "conv_wgrad_trp_kernel<6, 64"),
         ("head_dgrad", "head_dgrad_kernel"), ("head_bwd", "head_bwd_kernel"),
         ("conv1 wgrad", "conv1_wgrad_kernel"), ("adam", "adam_kernel"),
         ("bn2 bwd apply", "bn_bwd_apply_kernel"), ("conv3 wgrad", "conv_wgrad_trp_kernel<4, 32"))


def run(mode, steps):
    import torch
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl" if mode == "rccl" else "gloo", rank=0, world_size=1)
    import abd_amd
    from abd_amd import synth
    from abd_amd.models import smallcnn
    from abd_amd.pipeline import ResidentTrainer, attack_config, ultrasonic_trigger
    abd_amd.load_library()
    cfg = attack_config("ultrasonic")
    B, K = 512, 35
    waves, labels = synth.make_clips_torch(2048, cfg.sample_rate, cfg.length, K, seed=35, device=dev)
    torch.manual_seed(35)
    model = smallcnn(K, cfg.linear_features).to(dev)
    opt = torch.optim.Adam(model.parameters(), lr=1e-4)
    tr = ResidentTrainer(cfg, waves, labels, model, opt, B, trigger=ultrasonic_trigger(60, "mid", False), seed=35,
                         rank=0, world=1, collectives=True)
    red = tr.reducer
    if mode == "surrogate":
        def launch_fc():
            red.side.wait_event(red.event)
            with torch.cuda.stream(red.side):
                red.tail.mul_(1.0)     # stand-in for the collective's pass over the tail

        def finish():
            torch.cuda.current_stream().wait_stream(red.side)
            return red.flat
        red.launch_fc, red.finish = launch_fc, finish
    for _ in range(steps):
        tr.step()
    torch.cuda.synchronize()
    dist.destroy_process_group()
    print("done", mode, steps)


def report(d):
    f = sorted(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True))
    assert f, f"no kernel trace under {d}"
    rows = list(csv.DictReader(open(f[0])))
    ks = sorted(({"name": r["Kernel_Name"], "t0": int(r["Start_Timestamp"]), "t1": int(r["End_Timestamp"]),
                  "stream": r.get("Stream_Id"), "queue": r.get("Queue_Id")} for r in rows), key=lambda k: k["t0"])
    steps = [k for k in ks if "stft_mel" in k["name"]]
    side = [k for k in ks if "nccl" in k["name"].lower() or "rccl" in k["name"].lower()
            or ("elementwise" in k["name"] and "Mul" in k["name"])]
    print(f"{len(ks)} kernels, {len(steps)} steps (stft_mel launches), {len(side)} side-stream candidates")
    names = sorted({k["name"][:90] for k in side})
    for n in names:
        print("  side kernel:", n)
    out = []
    for i, s0 in enumerate(steps[:-1]):
        t0, t1 = s0["t0"], steps[i + 1]["t0"]
        inside = [k for k in ks if t0 <= k["t0"] < t1]
        sk = [k for k in side if t0 <= k["t0"] < t1]
        line = {"step": i, "step_us": (t1 - t0) / 1e3}
        for lab, pat in WATCH:
            m = [k for k in inside if pat in k["name"]]
            if m:
                line[lab] = ((m[0]["t0"] - t0) / 1e3, (m[-1]["t1"] - t0) / 1e3)
        line["side"] = [((k["t0"] - t0) / 1e3, (k["t1"] - t0) / 1e3, k["stream"]) for k in sk]
        conc = []
        for k in sk:   # kernels of other streams whose execution overlaps the side kernel's
            ov = [x["name"][:40] for x in inside if x is not k and x["t0"] < k["t1"] and x["t1"] > k["t0"]]
            conc.append(ov)
        line["concurrent_with"] = conc
        out.append(line)
    for line in out[-4:]:
        print(line)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", choices=["rccl", "surrogate"], default="rccl")
    ap.add_argument("--steps", type=int, default=12)
    ap.add_argument("--report", default=None)
    a = ap.parse_args()
    if a.report:
        report(a.report)
    else:
        run(a.mode, a.steps)


if __name__ == "__main__":
    main()
