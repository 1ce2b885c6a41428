"""Feasibility probe: the feature stage of batch k+1 on a side stream while batch k trains on the
main stream (double-buffered MFCC), against the sequential step.  bench.py's workload (ultrasonic,
B = 512).  Modes: seq | ovl (persistent STFT) | ovl with ABD_STFT_ONE_ITEM (a measurement-build knob, since removed) |
ovlcap (STFT grid capped by ABD_STFT_MAX_BLOCKS); PRIO=1 gives the main stream high priority."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import abd_amd  # noqa: E402
from abd_amd import synth  # noqa: E402
from abd_amd.models import smallcnn  # noqa: E402
from abd_amd.pipeline import ResidentTrainer, attack_config, ultrasonic_trigger  # noqa: E402

abd_amd.load_library()
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
cfg = attack_config("ultrasonic")
B, K = 512, 35
waves, labels = synth.make_clips_torch(8192, cfg.sample_rate, cfg.length, K, seed=35, device=dev)
torch.manual_seed(35)
model = smallcnn(K, cfg.linear_features).to(dev)
opt = torch.optim.Adam(model.parameters(), lr=1e-4)
tr = ResidentTrainer(cfg, waves, labels, model, opt, B, trigger=ultrasonic_trigger(60, "mid", False), seed=35,
                     gemm_precision="f32split")
mode = sys.argv[1] if len(sys.argv) > 1 else "seq"
steps = int(os.environ.get("STEPS", "100"))
prio = os.environ.get("PRIO") == "1"
lo, hi = torch.cuda.Stream.priority_range() if hasattr(torch.cuda.Stream, "priority_range") else (0, -1)
main = torch.cuda.Stream(priority=hi if prio else 0)
side = torch.cuda.Stream(priority=0)
xs = [torch.empty_like(tr.x), torch.empty_like(tr.x)]


def run(n):
    if mode == "seq":
        with torch.cuda.stream(main):
            for _ in range(n):
                b = tr._take_batch()
                tr._features(b, xs[0])
                tr._train(b, xs[0])
        return
    free = [torch.cuda.Event(), torch.cuda.Event()]
    ready = [torch.cuda.Event(), torch.cuda.Event()]
    for e in free:
        e.record(main)
    b = tr._take_batch()
    with torch.cuda.stream(side):
        tr._features(b, xs[0])
        ready[0].record(side)
    for k in range(n):
        cur = b
        if k + 1 < n:
            b = tr._take_batch()
            with torch.cuda.stream(side):
                side.wait_event(free[(k + 1) % 2])
                tr._features(b, xs[(k + 1) % 2])
                ready[(k + 1) % 2].record(side)
        with torch.cuda.stream(main):
            main.wait_event(ready[k % 2])
            tr._train(cur, xs[k % 2])
            free[k % 2].record(main)


run(10)
torch.cuda.synchronize()
t0 = time.perf_counter()
run(steps)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / steps
print(f"mode {mode} prio {int(prio)} env one_item={os.environ.get('ABD_STFT_ONE_ITEM')} "
      f"cap={os.environ.get('ABD_STFT_MAX_BLOCKS')}: {dt * 1e3:.4f} ms/step", flush=True)
