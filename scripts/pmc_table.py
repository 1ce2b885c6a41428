"""Per-kernel PMC table (last dispatch of each kernel) from rocprofv3 csv passes: python pmc_table.py DIR [substr...]"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
subs = sys.argv[2:]
vals = collections.defaultdict(dict)
dur = {}
for f in sorted(glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    name = {}
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        if subs and not any(s in k for s in subs):
            continue
        did = int(r["Dispatch_Id"])
        agg[did][r["Counter_Name"]] += float(r["Counter_Value"])
        name[did] = k
    last = {}
    for did in sorted(agg):
        last[name[did]] = agg[did]
    for k, v in last.items():
        vals[k].update(v)
for f in glob.glob(f"{d}/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        dur[k] = float(r["AverageNs"]) / 1e3
for k, v in sorted(vals.items(), key=lambda kv: -dur.get(kv[0], 0)):
    us = dur.get(k, 0)
    line = f"{k[:60]:60s} {us:8.1f}us"
    if "SQ_VALU_MFMA_BUSY_CYCLES" in v and "SQ_BUSY_CYCLES" in v and v["SQ_BUSY_CYCLES"]:
        line += f" mfma_busy/busy={v['SQ_VALU_MFMA_BUSY_CYCLES'] / (v['SQ_BUSY_CYCLES'] * 4 * 1):.3f}"
    if "SQ_WAVES" in v and v["SQ_WAVES"]:
        w = v["SQ_WAVES"]
        line += f" waves={w:.0f} valu/w={v.get('SQ_INSTS_VALU', 0) / w:.0f} lds/w={v.get('SQ_INSTS_LDS', 0) / w:.0f}"
        tot = v.get("SQ_WAIT_ANY", 0) + v.get("SQ_WAIT_INST_ANY", 0) + v.get("SQ_ACTIVE_INST_ANY", 0)
        if tot:
            line += f" wait={v.get('SQ_WAIT_ANY', 0) / tot:.2f} stall={v.get('SQ_WAIT_INST_ANY', 0) / tot:.2f} act={v.get('SQ_ACTIVE_INST_ANY', 0) / tot:.2f}"
    if "FETCH_SIZE" in v:
        line += f" fetchKB={v['FETCH_SIZE']:.0f}"
    if "WRITE_SIZE" in v:
        line += f" writeKB={v['WRITE_SIZE']:.0f}"
    if "SQ_LDS_BANK_CONFLICT" in v and v.get("SQ_LDS_IDX_ACTIVE"):
        line += f" ldsconf={v['SQ_LDS_BANK_CONFLICT'] / v['SQ_LDS_IDX_ACTIVE']:.2f}"
    print(line)
