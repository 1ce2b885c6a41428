"""Time the MFCC feature stage's two launches (stft_mel, db_dct) per launch at B = 512 ultrasonic
(HIP events, 40 launches after 5 warmup, REPS timings per process; the first is cold).  ABD_LIB
selects the library (A/B of two builds alternated on one box, scripts/gpu_r6_dbdct.sh)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import abd_amd  # noqa: E402
from abd_amd import _lib as L, features as F, synth  # noqa: E402

abd_amd.load_library()
dev = torch.device("cuda", 0)
B = int(os.environ.get("B", "512"))
c = F.MfccConfig.torchaudio(44100, 40, 1103, 441, 44100)
waves = synth.make_clips_torch(2048, c.sample_rate, c.length, 10, device=dev)[0]
rows = torch.randperm(2048, device=dev)[:B].to(torch.int32)
out = F.mfcc_batch(waves, c, rows=rows)
for _ in range(int(os.environ.get("REPS", "3"))):
    for _ in range(5):
        F.mfcc_batch(waves, c, rows=rows, out=out)
    torch.cuda.synchronize()
    with L.PhaseProfiler(["stft_mel", "db_dct"], max_records=128) as p:
        for _ in range(40):
            F.mfcc_batch(waves, c, rows=rows, out=out)
        torch.cuda.synchronize()
    r = p.result
    print("  ".join(f"{ph} {1e3 * r[ph][0] / r[ph][1]:.1f} us" for ph in ("stft_mel", "db_dct")), flush=True)
