"""Diagnostics: time the ultrasonic feature stage (B=512) with parts of stft_mel skipped."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import abd_amd  # noqa: E402
from abd_amd import features as F, synth, _lib as L  # noqa: E402

abd_amd.load_library()
dev = torch.device("cuda", 0)
B = int(os.environ.get("B", "512"))
cfgs = {"ultra": F.MfccConfig.torchaudio(44100, 40, 1103, 441, 44100),
        "n400": F.MfccConfig.torchaudio(16000, 40, 400, 160, 16000),
        "n2048": F.MfccConfig.torchaudio(16000, 13, 2048, 512, 16000)}
waves = {k: synth.make_clips_torch(2048, c.sample_rate, c.length, 10, device=dev)[0] for k, c in cfgs.items()}
rows = torch.randperm(2048, device=dev)[:B].to(torch.int32)
res = {}
for rnd in range(3):
    for name, c in cfgs.items():
        for ab in ("0", "1", "2", "4", "6", "7", "generic"):
            if ab == "generic":
                os.environ["ABD_GENERIC_FFT"] = "1"
                os.environ.pop("ABD_STFT_ABLATE", None)
            else:
                os.environ.pop("ABD_GENERIC_FFT", None)
                os.environ["ABD_STFT_ABLATE"] = ab
            F._PLANS.clear()
            out = F.mfcc_batch(waves[name], c, rows=rows)
            torch.cuda.synchronize()
            with L.PhaseProfiler(["stft_mel", "db_dct"], 256) as pr:
                for _ in range(10):
                    F.mfcc_batch(waves[name], c, rows=rows, out=out)
                torch.cuda.synchronize()
            ms = pr.result["stft_mel"][0] / pr.result["stft_mel"][1]
            res.setdefault((name, ab), []).append(ms)
for k, v in res.items():
    print(k, "stft_mel ms: min %.4f" % min(v), ["%.4f" % x for x in v])
