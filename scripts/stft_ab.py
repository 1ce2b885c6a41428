"""Time the feature stage (abd_mfcc_f32) per config: python scripts/stft_ab.py [iters]; ABD_LIB picks the .so.
Prints ms per launch (HIP events) and a checksum of the output (variants must agree)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import abd_amd  # noqa: E402
from abd_amd import features as F, synth  # noqa: E402

abd_amd.load_library()
dev = torch.device("cuda", 0)
iters = int(sys.argv[1]) if len(sys.argv) > 1 else 50
Bs = int(os.environ.get("B", "256"))   # the 16 kHz configs' batch (badnets / jingleback / daba / flowmur)
cfgs = {"ultra": (F.MfccConfig.torchaudio(44100, 40, 1103, 441, 44100), 512),
        "n400": (F.MfccConfig.torchaudio(16000, 40, 400, 160, 16000), Bs),
        "n2048": (F.MfccConfig.torchaudio(16000, 13, 2048, 512, 16000), Bs),
        "librosa": (F.MfccConfig.librosa(16000, 40, 16000), Bs)}
only = os.environ.get("CFGS")
for name, (c, B) in cfgs.items():
    if only and name not in only.split(","):
        continue
    waves = synth.make_clips_torch(2048, c.sample_rate, c.length, 10, device=dev)[0]
    rows = torch.randperm(2048, device=dev, generator=torch.Generator(device=dev).manual_seed(1))[:B].to(torch.int32)
    out = F.mfcc_batch(waves, c, rows=rows)
    for _ in range(5):
        F.mfcc_batch(waves, c, rows=rows, out=out)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(iters):
        F.mfcc_batch(waves, c, rows=rows, out=out)
    e1.record()
    torch.cuda.synchronize()
    print(f"{name:8s} B={B} {e0.elapsed_time(e1) / iters:.4f} ms/launch  checksum {float(out.double().sum()):.6f}",
          flush=True)
