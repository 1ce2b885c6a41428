#!/usr/bin/env python3
"""Per-mode summary of the convergence suite's printed per-epoch tables (pytest -s output of
tests/test_gpu_convergence.py): cells compared, cells where the GPU or reference value is below
99 % (not saturated), cells over the allowed gap, largest gap / allowed.
    python3 scripts/convergence_summary.py profiles/r5_convergence_tests.txt"""
import re
import sys


def main():
    cur, stats = None, {}
    for line in open(sys.argv[1]).read().splitlines():
        m = re.match(r"^(\w+) \[(.+)\]: per epoch, mean of", line)
        if m:
            cur = f"{m.group(1)} [{m.group(2)}]"
            stats[cur] = [0, 0, 0, 0.0]
            continue
        m = re.match(r"\s+epoch\s+\d+: ours\s+([-\d.]+)\s+ref\s+([-\d.]+) \+-\s+([-\d.]+)\s+gap\s+([-\d.]+) <=\s+([-\d.]+)",
                     line)
        if m and cur:
            o, r, _, g, a = map(float, m.groups())
            st = stats[cur]
            st[0] += 1
            st[1] += (r < 99 or o < 99)
            st[2] += g > a
            st[3] = max(st[3], g / a if a > 0 else 0.0)
    print(f"{'config [mode]':40s} cells  unsaturated  over  max gap/allowed")
    for k, v in stats.items():
        print(f"{k:40s} {v[0]:5d}  {v[1]:11d}  {v[2]:4d}  {v[3]:.2f}")


if __name__ == "__main__":
    main()
