"""Per-step host timing of a 2-rank gloo ResidentTrainer on one GPU (DP slowdown probe)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch, torch.distributed as dist
dist.init_process_group("gloo")
rank, world = dist.get_rank(), dist.get_world_size()
dev = torch.device("cuda", 0); torch.cuda.set_device(dev)
import abd_amd
from abd_amd import synth, parallel_dp as DP, training as T
from abd_amd.models import smallcnn
from abd_amd.pipeline import ResidentTrainer, attack_config, ultrasonic_trigger
abd_amd.load_library()
cfg = attack_config("ultrasonic")
waves, labels = synth.make_clips_torch(2048, cfg.sample_rate, cfg.length, 35, seed=35 + rank, device=dev)
torch.manual_seed(35)
model = smallcnn(35, cfg.linear_features).to(dev)
opt = torch.optim.Adam(model.parameters(), lr=1e-4)
tr = ResidentTrainer(cfg, waves, labels, model, opt, 512, trigger=ultrasonic_trigger(60, "mid", False), seed=35,
                     rank=rank, world=world, overlap_features=os.environ.get("OVL", "0") == "1")
for i in range(8):
    torch.cuda.synchronize(); dist.barrier()
    t0 = time.perf_counter()
    batch = tr._take_batch() if not tr.overlap else None
    if batch is not None:
        tr._features(batch, tr.x); torch.cuda.synchronize(); t1 = time.perf_counter()
        _, lab, ind, _, _ = batch
        T.train_step(tr.model, tr.x, lab, ind, tr.adam, tr.metrics, do_update=False, grad_scale=0.5,
                     fc_grads_event=tr.reducer.event_ptr())
        torch.cuda.synchronize(); t2 = time.perf_counter()
        tr.reducer.launch_fc(); t3 = time.perf_counter()
        tr.reducer.finish(); t4 = time.perf_counter()
        torch.cuda.synchronize(); t5 = time.perf_counter()
        T.apply_adam(tr.model, tr.adam, dev); torch.cuda.synchronize(); t6 = time.perf_counter()
        print(f"rank{rank} step{i} feat {1e3*(t1-t0):.1f} train {1e3*(t2-t1):.1f} launch {1e3*(t3-t2):.1f} "
              f"finish {1e3*(t4-t3):.1f} sync {1e3*(t5-t4):.1f} adam {1e3*(t6-t5):.1f}", flush=True)
    else:
        tr.step(); torch.cuda.synchronize(); print(f"rank{rank} step{i} total {1e3*(time.perf_counter()-t0):.1f}", flush=True)
# free-running like bench.py (no per-step sync)
torch.cuda.synchronize(); dist.barrier()
ts = [time.perf_counter()]
for i in range(12):
    tr.step()
    ts.append(time.perf_counter())
torch.cuda.synchronize(); ts.append(time.perf_counter())
print(f"rank{rank} free " + " ".join(f"{1e3*(b-a):.1f}" for a, b in zip(ts, ts[1:])), flush=True)
dist.destroy_process_group()
