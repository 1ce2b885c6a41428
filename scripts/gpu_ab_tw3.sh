#!/bin/bash
# A/B: STFT pass-3 twiddles from the table (-DABD_TW3_TABLE) vs base + powers, scalar-FP32 build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-ab_tw3}; mkdir -p $O
for r in 1 2; do for v in default tw3; do
  L=""; [ $v != default ] && L=$PWD/audio-backdoor-attack_amd/libabd_$v.so
  ABD_LIB=${L:-$PWD/audio-backdoor-attack_amd/libabd.so} timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu --dropin-batches 0 > $O/$v$r.json 2> $O/$v$r.err || { tail $O/$v$r.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/$v$r.json').read().strip().splitlines()[-1]); p=d.get('phases_ms_per_launch') or {}
print('$v$r', d['ms_per_step'], p.get('stft_mel'), p.get('db_dct'))"
done; done
