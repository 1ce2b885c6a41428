"""Summarise rocprofv3 PMC csv passes for one kernel (last dispatch): python pmc_summary.py DIR SUBSTR"""
import collections
import csv
import glob
import sys

d, sub = sys.argv[1], sys.argv[2]
vals = {}
for f in sorted(glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    meta = {}
    for r in csv.DictReader(open(f)):
        if sub not in r["Kernel_Name"]:
            continue
        agg[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
        meta = {k: r[k] for k in ("Grid_Size", "Workgroup_Size", "LDS_Block_Size", "VGPR_Count", "SGPR_Count")}
    if agg:
        vals.update(agg[max(agg)])
print(meta)
for k in sorted(vals):
    print(f"{k:28s} {vals[k]:.4g}")
w = vals.get("SQ_WAVES", 0)
if w:
    print("VALU/wave %.0f  LDS/wave %.0f  wave-life us %.1f" % (vals["SQ_INSTS_VALU"] / w, vals["SQ_INSTS_LDS"] / w,
                                                              4 * vals["SQ_WAVE_CYCLES"] / w / 2.4e3))
    print("VALU issue-bound us (256 CUs, 1 wave-instr/clk/CU): %.1f" % (vals["SQ_INSTS_VALU"] / 256 / 2.4e3))
