"""Drive only the MFCC feature stage (for rocprofv3 PMC passes): CFG=ultra|n400|n2048, ITERS launches."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import abd_amd  # noqa: E402
from abd_amd import features as F, synth  # noqa: E402

abd_amd.load_library()
dev = torch.device("cuda", 0)
B = int(os.environ.get("B", "512"))
name = os.environ.get("CFG", "ultra")
c = {"ultra": F.MfccConfig.torchaudio(44100, 40, 1103, 441, 44100),
     "n400": F.MfccConfig.torchaudio(16000, 40, 400, 160, 16000),
     "n2048": F.MfccConfig.torchaudio(16000, 13, 2048, 512, 16000)}[name]
waves = synth.make_clips_torch(2048, c.sample_rate, c.length, 10, device=dev)[0]
rows = torch.randperm(2048, device=dev)[:B].to(torch.int32)
out = F.mfcc_batch(waves, c, rows=rows)
for _ in range(int(os.environ.get("ITERS", "5"))):
    F.mfcc_batch(waves, c, rows=rows, out=out)
torch.cuda.synchronize()
print("done", name, tuple(out.shape))
