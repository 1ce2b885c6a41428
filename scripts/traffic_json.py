"""HBM bytes per launch of the bench phases from rocprofv3 FETCH_SIZE / WRITE_SIZE passes.

    python scripts/traffic_json.py gpurun_out/<tag> profiles/<name>_traffic.json

Corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950
FETCH_SIZE reports half the bytes of wide (16 B/lane) coalesced reads, so it is doubled; WRITE_SIZE
is exact for 16-B stores.

Kernels are matched by their EXACT name (template arguments included, argument list dropped) and,
for a kernel that runs more than once per step (bn_bwd_apply_kernel: BN3 then BN2), by its
occurrence within the LAST step of the profiled run (the dispatches after the last STFT launch).
The output records the sha1 of the libabd sources it was measured on (``csrc_sha1``), read from
``<run dir>/csrc_sha1.txt`` (written on the GPU box by scripts/round_full.sh before it profiles);
a run directory without that file is refused unless ``--tree-sha`` says the current tree IS the
measured one.  bench.py only uses a traffic file whose hash matches the sources it runs, and names
that file per phase.
"""
import collections
import csv
import glob
import hashlib
import json
import os
import re
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# phase -> candidate (exact kernel, occurrence within one step); the first candidate present is used
PHASE_KERNELS = {
    "stft_mel": [("stft_mel_fast_kernel<2304, 1103, 16, 12, 12, 1, true, 8>", 0),
                 ("stft_mel_fast_kernel<2304, 1103, 16, 12, 12, 1, true>", 0)],
    "db_dct": [("db_dct_mfma_kernel<3>", 0)],
    "conv1_stats": [("conv1_stats_fold_kernel", 0), ("conv1_stats_kernel", 0)],
    "conv2_fwd": [("conv_ws_spec_kernel<1, 2, 3>", 0), ("conv_ws_spec_kernel<1, 2, 1>", 0), ("conv_ws_spec_kernel<1, 2>", 0), ("conv_ws_pre_kernel<1, 2>", 0), ("conv_ws_dma_kernel<1, 3, 2, false>", 0),
                  ("conv_ws_dma_kernel<1, 1, 2, true>", 0), ("conv_ws_dma_kernel<1, 3, 2>", 0), ("conv_ws_dma_kernel<1, 1, 2>", 0),
                  ("conv_ws_dma_kernel<1, 3>", 0), ("conv_ws_dma_kernel<1, 1>", 0),
                  ("conv_ws_dma_kernel<3>", 0), ("conv_ws_dma_kernel<1>", 0),
                  ("conv_ws_split_kernel<1, 2, 64, 1, 8, 8, 3, false, true>", 0),
                  ("conv_ws_split_kernel<1, 2, 64, 1, 8, 8, 1, true, true>", 0),
                  ("conv_ws_split_kernel<1, 2, 64, 1, 8, 8, 3, false>", 0),
                  ("conv_ws_split_kernel<1, 2, 64, 1, 8, 8, 1, true>", 0),
                  ("conv_ws_split_kernel<1, 2, 64, 1, 8, 8, 1, false>", 0)],
    "bn2_pool": [("bn_pool_fwd_kernel", 0)],
    "conv3_fwd": [("conv_ws_spec_kernel<1, 1, 3>", 0), ("conv_ws_spec_kernel<1, 1>", 0), ("conv_ws_pre_kernel<1, 1>", 0), ("conv_ws_dma_kernel<1, 3, 1, false>", 0),
                  ("conv_ws_dma_kernel<1, 1, 1, false>", 0), ("conv_ws_dma_kernel<1, 3, 1>", 0), ("conv_ws_dma_kernel<1, 1, 1>", 0),
                  ("conv_ws_split_kernel<1, 1, 64, 1, 4, 8, 3, false, true>", 0),
                  ("conv_ws_split_kernel<1, 1, 64, 1, 4, 8, 1, false, true>", 0),
                  ("conv_ws_split_kernel<1, 1, 64, 1, 4, 8, 3, false>", 0),
                  ("conv_ws_split_kernel<1, 1, 64, 1, 4, 8, 1, false>", 0)],
    "bn3_pool_dropout": [("bn_pool_fwd_kernel", 1)],
    "head_fwd": [("head_fwd_kernel<4>", 0), ("head_fwd_kernel<8>", 0), ("head_fwd_kernel", 0)],
    "head_mid": [("head_row_kernel", 0), ("head_mid_kernel", 0)],
    "head_dgrad": [("head_dgrad_kernel", 0)],
    "head_bwd": [("head_bwd_kernel", 0)],
    "fc1_fwd": [("gemm_nt_kernel<128, 4, 1, 32>", 0)],
    "fc1_wgrad": [("gemm_tn_kernel<128, 128>", 0)],
    "fc1_dgrad": [("gemm_nt_kernel<32, 3, 1, 32>", 0)],
    # bn_bwd_apply_kernel runs BN3 then BN2 (round-2 head) or BN2 alone (fused head): count from the end
    "bn3_bwd": [("bn_bwd_apply_kernel", -2)],
    "bn2_bwd": [("bn_bwd_apply_kernel", -1)],
    "conv3_wgrad": [("conv_wgrad_trp_kernel<4, 32, 2, 4, 3, false>", 0), ("conv_wgrad_trp_kernel<4, 32, 2, 4, 1, false>", 0)],
    "conv3_dgrad": [("conv_ws_split_kernel<0, 2, 32, 1, 4, 8, 3, false, false>", 0),
                    ("conv_ws_split_kernel<0, 2, 32, 1, 4, 8, 1, false, false>", 0),
                    ("conv_ws_split_kernel<0, 2, 32, 1, 4, 8, 3, false>", 0),
                    ("conv_ws_split_kernel<0, 2, 32, 1, 4, 8, 1, false>", 0)],
    "conv2_wgrad": [("conv_wgrad_trp_kernel<6, 64, 5, 11, 3, false>", 0),
                    ("conv_wgrad_trp_kernel<6, 64, 5, 11, 1, true>", 0)],
    "conv2_dgrad": [("conv_ws_spec_kernel<0, 2, 3>", 0), ("conv_ws_spec_kernel<0, 2, 1>", 0), ("conv_ws_spec_kernel<0, 2>", 0), ("conv_ws_pre_kernel<0, 2>", 0), ("conv_ws_dma_kernel<0, 1, 2, true>", 0),
                    ("conv_ws_split_kernel<0, 2, 64, 1, 8, 8, 3, false, false>", 0),
                    ("conv_ws_split_kernel<0, 2, 64, 1, 8, 8, 1, true, false>", 0),
                    ("conv_ws_split_kernel<0, 2, 64, 1, 8, 8, 3, false>", 0),
                    ("conv_ws_split_kernel<0, 2, 64, 1, 8, 8, 1, true>", 0)],
    "conv1_bwd_wgrad": [("conv1_wgrad_kernel<true>", 0)],
}
STEP_START = "stft_mel_fast_kernel<"


# the sources every bench-step kernel is compiled from (the feature stage, the train step, the fused
# head included by smallcnn.hip, the shared headers); effects / resample / DABA / the C-ABI glue run
# no kernel of the bench step, so editing them does not invalidate a traffic measurement
BENCH_SOURCES = ("mfcc.hip", "smallcnn.hip", "fc_head.inc", "abd_common.h", "prof.h", "prof.cpp")


def csrc_sha1(root=HERE):
    """sha1 over the bench step's libabd sources (name + bytes, sorted): identifies the code a
    measurement belongs to."""
    h = hashlib.sha1()
    d = os.path.join(root, "audio-backdoor-attack_amd", "csrc")
    for f in sorted(os.listdir(d)):
        if f in BENCH_SOURCES:
            h.update(f.encode())
            h.update(open(os.path.join(d, f), "rb").read())
    return h.hexdigest()


def kernel_key(name):
    k = name.replace("void ", "").replace("(anonymous namespace)::", "")
    return k[:k.index("(")] if "(" in k else k


def last_step(d, counter):
    """[(kernel key, value)] of the dispatches after the last STFT launch, in dispatch order."""
    rows = []
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        agg = collections.defaultdict(float)
        name = {}
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            did = int(r["Dispatch_Id"])
            agg[did] += float(r["Counter_Value"])
            name[did] = kernel_key(r["Kernel_Name"])
        rows += [(did, name[did], agg[did]) for did in agg]
    rows.sort()
    starts = [i for i, (_, k, _) in enumerate(rows) if k.startswith(STEP_START)]
    if not starts:
        return []
    return [(k, v) for _, k, v in rows[starts[-1]:]]


def pick(step, cands):
    """First candidate present: (kernel, occurrence, value); a negative occurrence counts from the end."""
    for key, occ in cands:
        hits = [v for k, v in step if k == key]
        if (occ >= 0 and len(hits) > occ) or (occ < 0 and len(hits) >= -occ):
            return key, occ, hits[occ]
    return None


def main():
    if len(sys.argv) == 2 and sys.argv[1] == "--print-sha":
        print(csrc_sha1())
        return
    args = [a for a in sys.argv[1:] if a != "--tree-sha"]
    d, dst = args[0], args[1]
    shaf = os.path.join(d, "csrc_sha1.txt")
    if os.path.exists(shaf):
        sha = open(shaf).read().strip()
    elif "--tree-sha" in sys.argv:
        sha = csrc_sha1()
    else:
        sys.exit(f"{shaf} missing: the sources this run measured are unknown (pass --tree-sha if they are "
                 "the current tree's)")
    fetch, write = last_step(d, "FETCH_SIZE"), last_step(d, "WRITE_SIZE")
    res = {"source": d, "csrc_sha1": sha,
           "correction": "FETCH_SIZE x2 (gfx950 wide reads), KiB -> bytes; last profiled step", "bytes_per_launch": {},
           "detail": {}}
    for ph, cands in PHASE_KERNELS.items():
        f, w = pick(fetch, cands), pick(write, cands)
        if f is None or w is None:
            continue
        rb, wb = 2 * f[2] * 1024, w[2] * 1024
        res["bytes_per_launch"][ph] = round(rb + wb)
        res["detail"][ph] = {"kernel": f[0], "occurrence": f[1], "read_bytes": round(rb), "write_bytes": round(wb)}
    # VALU wave-instructions per launch (summed over the chip), when the run has an SQ_INSTS_VALU pass
    # (round_full.sh's p_sq): bench.py prices stft_mel against the VALU issue limit with it
    valu = last_step(d, "SQ_INSTS_VALU")
    if valu:
        res["valu_insts_per_launch"] = {}
        for ph, cands in PHASE_KERNELS.items():
            v = pick(valu, cands)
            if v is not None:
                res["valu_insts_per_launch"][ph] = round(v[2])
    json.dump(res, open(dst, "w"), indent=1)
    print(json.dumps(res["bytes_per_launch"]))


if __name__ == "__main__":
    main()
