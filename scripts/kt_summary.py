#!/usr/bin/env python3
"""Per-step kernel timeline of a rocprofv3 kernel trace (scripts/kt_quick.sh output).

    python3 scripts/kt_summary.py gpurun_out/ktq_TAG [STEP_MARKER]

Steps are delimited by the feature-stage launch (STEP_MARKER, default "stft_mel").  Prints, for the
last full steps, each kernel's start offset, duration and the idle gap before it, then the step's
busy time (sum of kernel durations) against its span.
"""
import csv
import glob
import os
import sys


def main():
    d = sys.argv[1]
    mark = sys.argv[2] if len(sys.argv) > 2 else "stft_mel"
    f = sorted(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True))[0]
    ks = sorted(({"n": r["Kernel_Name"], "t0": int(r["Start_Timestamp"]), "t1": int(r["End_Timestamp"])}
                 for r in csv.DictReader(open(f))), key=lambda k: k["t0"])
    st = [i for i, k in enumerate(ks) if mark in k["n"]]
    spans = []
    for a, b in zip(st[:-1], st[1:]):
        seg = ks[a:b]
        span = (ks[b]["t0"] - seg[0]["t0"]) / 1e3
        busy = sum(k["t1"] - k["t0"] for k in seg) / 1e3
        spans.append((span, busy, seg, ks[b]["t0"]))
    # steady-state steps: drop profiling / warmup outliers by taking the median-span steps
    good = sorted(spans, key=lambda s: s[0])[len(spans) // 4: len(spans) // 4 + 3]
    for span, busy, seg, tend in good[:1]:
        t0 = seg[0]["t0"]
        prev = t0
        for k in seg:
            nm = k["n"].replace("(anonymous namespace)::", "")
            nm = nm.split("(")[0] if not nm.startswith("void at::") else nm[:60]
            print(f"{(k['t0'] - t0) / 1e3:8.1f} {(k['t1'] - k['t0']) / 1e3:7.1f} gap {(k['t0'] - prev) / 1e3:5.1f}  {nm[:80]}")
            prev = k["t1"]
        print(f"  tail gap {(tend - prev) / 1e3:.1f}")
    for span, busy, seg, _ in good:
        print(f"step span {span:.1f} us, busy {busy:.1f} us, {len(seg)} kernels, idle {span - busy:.1f} us")


if __name__ == "__main__":
    main()
