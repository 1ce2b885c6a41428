"""Is the step host-bound?  Times the host's enqueue of N train steps (no sync) against the device
time of the same steps (sync after).  python scripts/host_probe.py [N] [attack] [batch]
(default: the headline, ultrasonic at B = 512)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import abd_amd  # noqa: E402
from abd_amd import synth  # noqa: E402
from abd_amd.models import smallcnn  # noqa: E402
from abd_amd.pipeline import ResidentTrainer, attack_config, ultrasonic_trigger  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    attack = sys.argv[2] if len(sys.argv) > 2 else "ultrasonic"
    batch = int(sys.argv[3]) if len(sys.argv) > 3 else 512
    dev = torch.device("cuda", 0)
    abd_amd.load_library()
    cfg = attack_config(attack)
    K = 35 if attack == "ultrasonic" else 10
    waves, labels = synth.make_clips_torch(8192, cfg.sample_rate, cfg.length, K, seed=35, device=dev)
    trigger = None
    if attack == "ultrasonic":
        trigger = ultrasonic_trigger(60, "mid", False)
    elif attack == "flowmur":   # as bench.py: a fixed learned-trigger stand-in, target-class clips present
        import numpy as np
        labels[: 8192 // 4] = cfg.target_label
        trigger = (0.05 * np.random.default_rng(1).standard_normal(8000)).astype(np.float32)
    torch.manual_seed(35)
    model = smallcnn(K, cfg.linear_features).to(dev)
    opt = torch.optim.Adam(model.parameters(), lr=1e-4)
    tr = ResidentTrainer(cfg, waves, labels, model, opt, batch, trigger=trigger, seed=35)
    for _ in range(20):
        tr.step()
    torch.cuda.synchronize()
    for rep in range(3):
        t0 = time.perf_counter()
        for _ in range(n):
            tr.step()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"rep {rep}: host enqueue {1e3 * (t1 - t0) / n:.4f} ms/step, wall {1e3 * (t2 - t0) / n:.4f} ms/step",
              flush=True)
    # host cost of one step with the device idle (sync before each)
    ts = []
    for _ in range(50):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        tr.step()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    print(f"idle-device host cost per step: median {1e3 * ts[len(ts) // 2]:.4f} ms", flush=True)


if __name__ == "__main__":
    main()
