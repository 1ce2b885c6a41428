#!/bin/bash
# Same-box A/B of the pre-split routing levels (ABD_WS_PRE 0..3), three alternations, default DMA mode.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-ab_pre}; mkdir -p $O
for r in 1 2 3; do for v in pre0 pre1 pre2 default; do
  L=$PWD/audio-backdoor-attack_amd/libabd.so; [ $v != default ] && L=$PWD/audio-backdoor-attack_amd/libabd_$v.so
  ABD_LIB=$L timeout -k 10 300 python bench.py --steps 300 --warmup 30 --no-cpu --dropin-batches 0 > $O/$v$r.json 2> $O/$v$r.err || { tail $O/$v$r.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/$v$r.json').read().strip().splitlines()[-1]); p=d.get('phases_ms_per_launch') or {}
print('$v$r', d['ms_per_step'], d['ms_per_step_window_median'], {k: round(p[k], 4) for k in ('conv2_fwd','conv2_dgrad','conv3_fwd') if k in p})"
done; done
