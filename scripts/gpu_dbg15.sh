#!/bin/bash
# Packed-FP32-free build vs default: bench (single process) and the sharing probe on the full nopk build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-dbg15}; mkdir -p $O
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu --dropin-batches 0 > $O/bench_default.json 2> $O/bench_default.err || { tail $O/bench_default.err; exit 1; }
ABD_LIB=$PWD/audio-backdoor-attack_amd/libabd_nopk.so timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu --dropin-batches 0 > $O/bench_nopk.json 2> $O/bench_nopk.err || { tail $O/bench_nopk.err; exit 1; }
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu --dropin-batches 0 > $O/bench_default2.json 2> $O/bench_default2.err || { tail $O/bench_default2.err; exit 1; }
for f in default nopk default2; do python3 -c "
import json,sys; d=json.loads(open('$O/bench_$f.json').read().strip().splitlines()[-1]); p=d.get('phases_ms_per_launch') or {}
print('$f', d['value'], d['ms_per_step'], {k: round(v,4) for k,v in p.items()})"; done
for i in 1 2 3 4; do ABD_LIB=$PWD/audio-backdoor-attack_amd/libabd_nopk.so ABD_WS_DMA=0 timeout -k 10 170 python scripts/share_buffers.py f32split 2 60 32 >> $O/share.txt 2>&1 || { tail $O/share.txt; exit 1; }; done
grep "^(" $O/share.txt | cut -c1-200
