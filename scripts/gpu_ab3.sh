#!/bin/bash
# Same-box A/B of library variants, three alternations of 300 steps (libabd_<v>.so; "default" = libabd.so).
# Usage: bash scripts/gpu_ab3.sh TAG v1 v2 ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=$1; shift
O=gpurun_out/$T; mkdir -p $O
for r in 1 2 3; do for v in "$@"; do
  L=$PWD/audio-backdoor-attack_amd/libabd.so; [ $v != default ] && L=$PWD/audio-backdoor-attack_amd/libabd_$v.so
  ABD_LIB=$L timeout -k 10 300 python bench.py --steps 300 --warmup 30 --no-cpu --dropin-batches 0 > $O/$v$r.json 2> $O/$v$r.err || { tail $O/$v$r.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/$v$r.json').read().strip().splitlines()[-1]); p=d.get('phases_ms_per_launch') or {}
print('$v$r', d['ms_per_step'], d['ms_per_step_window_median'], round(sum(p.values()), 4), {k: round(p[k], 4) for k in ('conv2_fwd','conv2_dgrad','conv3_fwd','bn2_pool','conv1_stats') if k in p})"
done; done
