"""row_scale_kernel alone (FlowMur SNR mix): python3 scripts/row_scale_probe.py [poison_fraction]; run under
rocprofv3 --kernel-trace --stats to read the kernel's duration at B = 256, 16 kHz x 1 s rows."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import abd_amd  # noqa: E402
from abd_amd import _lib as L, features as F  # noqa: E402

abd_amd.load_library()
dev = torch.device("cuda", 0)
frac = float(sys.argv[1]) if len(sys.argv) > 1 else 0.1
B, N, Lc = 256, 2048, 16000
g = torch.Generator(device=dev).manual_seed(1)
waves = torch.randn(N, Lc, device=dev, generator=g) * 0.1
rows = torch.randperm(N, device=dev, generator=g)[:B].to(torch.int32)
pois = (torch.rand(B, device=dev, generator=g) < frac).to(torch.uint8)
trig = torch.randn(8000, device=dev, generator=g) * 0.05
pos = torch.randint(0, Lc - 8000, (B,), device=dev, generator=g, dtype=torch.int32)
inj = F.Injection(mode=L.INJECT_SNR_WINDOW, trigger=trig, poison=pois, position=pos, snr_db=30.0)
for _ in range(50):
    F.inject_waveform(waves, Lc, inj, rows=rows)
torch.cuda.synchronize()
print("poisoned rows", int(pois.sum()))
