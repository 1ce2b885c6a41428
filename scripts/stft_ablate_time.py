"""Time the MFCC feature stage's stft_mel launch under ABD_STFT_ABLATE bits (a library built with
-DABD_STFT_ABLATE_BUILD, selected by ABD_LIB): 0 full, 1 no sample/chirp loads, 2 no FFTs, 4 no
power/mel, and their sums.  Results are garbage; only the launch times are read (HIP events)."""
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
for bits in [int(b) for b in os.environ.get("BITS", "0,1,2,4,6,7,0").split(",")]:
    os.environ["ABD_STFT_ABLATE"] = str(bits)
    for _ in range(5):
        F.mfcc_batch(waves, c, rows=rows, out=out)
    torch.cuda.synchronize()
    with L.PhaseProfiler(["stft_mel"], max_records=64) as p:
        for _ in range(40):
            F.mfcc_batch(waves, c, rows=rows, out=out)
        torch.cuda.synchronize()
    ms, n = p.result["stft_mel"]
    print(f"ablate {bits}: stft_mel {1e3 * ms / n:.1f} us ({n} launches)", flush=True)
