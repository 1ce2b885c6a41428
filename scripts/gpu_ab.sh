#!/bin/bash
# A/B of library variants (libabd_<v>.so, "default" = libabd.so): bench phases, two alternations.
# Usage: bash scripts/gpu_ab.sh TAG PHASE v1 v2 ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=$1; PH=$2; shift 2
O=gpurun_out/$T; mkdir -p $O
for r in 1 2; do for v in "$@"; do
  L=$PWD/audio-backdoor-attack_amd/libabd.so; [ $v != default ] && L=$PWD/audio-backdoor-attack_amd/libabd_$v.so
  ABD_LIB=$L timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu --dropin-batches 0 > $O/$v$r.json 2> $O/$v$r.err || { tail $O/$v$r.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/$v$r.json').read().strip().splitlines()[-1]); p=d.get('phases_ms_per_launch') or {}
print('$v$r', d['ms_per_step'], {k: round(p[k], 4) for k in '$PH'.split(',') if k in p})"
done; done
