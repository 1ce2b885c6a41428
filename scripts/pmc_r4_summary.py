#!/usr/bin/env python3
"""Per-kernel counter tables from a pmc_r4.sh run: python scripts/pmc_r4_summary.py RUN_DIR OUT_DIR
(conv: the train-step kernels of one profiled bench step; stft: the Bluestein STFT alone).  FETCH_SIZE
is doubled (MI355X_MICROARCH.md, gfx950 wide reads) and both byte counters converted from KiB."""
import collections
import csv
import glob
import os
import sys

run, out = sys.argv[1], sys.argv[2]
KERNELS = {
    "conv": ["conv_ws_spec_kernel<1, 2", "conv_ws_spec_kernel<0, 2", "conv_ws_spec_kernel<1, 1",
             "conv_ws_pre_kernel<1, 2>", "conv_ws_pre_kernel<0, 2>", "conv_ws_pre_kernel<1, 1>",
             "conv_ws_dma_kernel<1, 3, 2", "conv_ws_split_kernel<0, 2, 64", "conv_wgrad_trp_kernel<6, 64",
             "conv_ws_dma_kernel<1, 3, 1", "conv_ws_split_kernel<0, 2, 32", "conv_wgrad_trp_kernel<4, 32",
             "conv1_wgrad_kernel", "conv1_stats_fold_kernel", "bn_bwd_apply_kernel", "bn_pool_fwd_kernel",
             "head_fwd_kernel", "head_row_kernel", "head_dgrad_kernel", "head_bwd_kernel"],
    "stft": ["stft_mel_fast_kernel", "db_dct_mfma_kernel"],
}


def counters(prefix, sub):
    vals, meta = {}, {}
    for f in sorted(glob.glob(os.path.join(run, f"{prefix}_*", "**", "*counter_collection.csv"), recursive=True)):
        agg = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in csv.DictReader(open(f)):
            if sub not in r["Kernel_Name"]:
                continue
            agg[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
            meta = {k: r[k] for k in ("Grid_Size", "Workgroup_Size", "LDS_Block_Size", "VGPR_Count")}
        if agg:
            vals.update(agg[max(agg)])   # the last dispatch: one bench step / one STFT launch
    return vals, meta


os.makedirs(out, exist_ok=True)
for prefix, subs in KERNELS.items():
    lines = []
    for sub in subs:
        v, meta = counters(prefix, sub)
        if not v:
            continue
        lines.append(f"### {sub}   {meta}")
        for k in sorted(v):
            lines.append(f"{k:34s} {v[k]:.4g}")
        if v.get("SQ_WAVE_CYCLES"):
            lines.append(f"{'= wait fraction (SQ_WAIT_ANY / SQ_WAVE_CYCLES)':34s} {v['SQ_WAIT_ANY'] / v['SQ_WAVE_CYCLES']:.3f}")
        if v.get("SQ_INSTS_LDS") and "SQ_LDS_BANK_CONFLICT" in v:
            lines.append(f"{'= bank-conflict cycles per LDS instr':34s} {v['SQ_LDS_BANK_CONFLICT'] / v['SQ_INSTS_LDS']:.3f}")
        if "FETCH_SIZE" in v:
            lines.append(f"{'= HBM read MB (FETCH_SIZE x2)':34s} {v['FETCH_SIZE'] * 2 * 1024 / 1e6:.1f}")
        if "WRITE_SIZE" in v:
            lines.append(f"{'= HBM write MB':34s} {v['WRITE_SIZE'] * 1024 / 1e6:.1f}")
        lines.append("")
    with open(os.path.join(out, f"{prefix}_counters.txt"), "w") as fh:
        fh.write("\n".join(lines) + "\n")
    print(prefix, len(lines), "lines")
