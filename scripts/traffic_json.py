"""HBM bytes per launch for the bench phases from rocprofv3 FETCH_SIZE / WRITE_SIZE passes.

    python scripts/traffic_json.py gpurun_out/<tag> profiles/<name>_traffic.json

Corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE and WRITE_SIZE are in KiB;
on gfx950 FETCH_SIZE reports half the bytes of wide (16 B/lane) coalesced reads, so it is
doubled; WRITE_SIZE is exact for 16-B stores.  The last dispatch of each kernel in the
profiled bench run is used (steady state).  Kernels shared by two phases (gemm_nt<64,0>
runs conv3 then conv2 data gradients) resolve to the later one, conv2.  A phase lists the
fp32 kernel and the f32split kernel; the profiled run uses one of them.
"""
import collections
import csv
import glob
import json
import sys

PHASE_KERNELS = {
    "stft_mel": "stft_mel_fast_kernel<2304, 1103",
    "db_dct": ("db_dct_lds_kernel", "db_dct_mfma_kernel"),
    "conv2_fwd": ("gemm_nt_kernel<64, 1, 1>", "gemm_nt_bf16_kernel<64, 1, 32, 3, 1>", "conv_ws_split_kernel<1"),
    "conv2_dgrad": ("gemm_nt_kernel<64, 0, 1>", "gemm_nt_bf16_kernel<64, 0, 32, 3, 1>", "conv_ws_split_kernel<0"),
    "conv2_wgrad": "conv_wgrad_rows_kernel<64, 64>",
    "conv1_bwd_wgrad": "conv1_wgrad_kernel",
    "bn2_bwd": "bn_bwd_apply_kernel",
}


def last_dispatch(d, counter):
    out = {}
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        agg = collections.defaultdict(float)
        name = {}
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            did = int(r["Dispatch_Id"])
            agg[did] += float(r["Counter_Value"])
            name[did] = r["Kernel_Name"]
        for did in sorted(agg):
            out[name[did]] = agg[did]
    return out


def main():
    d, dst = sys.argv[1], sys.argv[2]
    fetch = last_dispatch(d, "FETCH_SIZE")
    write = last_dispatch(d, "WRITE_SIZE")
    res = {"source": d, "correction": "FETCH_SIZE x2 (gfx950 wide reads), KiB -> bytes", "bytes_per_launch": {},
           "detail": {}}
    for ph, subs in PHASE_KERNELS.items():
        subs = subs if isinstance(subs, tuple) else (subs,)   # fp32 kernel, f32split kernel
        fk = [v for k, v in fetch.items() if any(x in k for x in subs)]
        wk = [v for k, v in write.items() if any(x in k for x in subs)]
        if not fk or not wk:
            continue
        rb, wb = 2 * fk[-1] * 1024, wk[-1] * 1024
        res["bytes_per_launch"][ph] = round(rb + wb)
        res["detail"][ph] = {"read_bytes": round(rb), "write_bytes": round(wb)}
    json.dump(res, open(dst, "w"), indent=1)
    print(json.dumps(res["bytes_per_launch"]))


if __name__ == "__main__":
    main()
