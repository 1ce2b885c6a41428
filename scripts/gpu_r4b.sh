#!/bin/bash
# r4_v2: DP debug probes, conv probe (default vs spread DMA), then the parity suite + smoke + bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r4_v2}; mkdir -p $O
timeout -k 10 200 python scripts/dp_debug.py > $O/dp_debug.txt 2>&1 || { tail -20 $O/dp_debug.txt; exit 1; }
grep -v "Warning\|socket\|Gloo\|amdgpu.ids" $O/dp_debug.txt | tail -12
timeout -k 10 300 python scripts/dp_overlap_debug.py f32 f32split > $O/overlap.txt 2>&1 || { tail -20 $O/overlap.txt; exit 1; }
grep -v "Warning\|socket\|Gloo\|amdgpu.ids" $O/overlap.txt | tail -8
for lib in libabd.so libabd_spread.so libabd.so libabd_spread.so; do
  ABD_LIB=$PWD/audio-backdoor-attack_amd/$lib timeout -k 10 120 python scripts/conv_probe.py --tag $lib >> $O/conv.jsonl 2>> $O/conv.err || { tail -20 $O/conv.err; exit 1; }
done
python3 -c "
import json
for l in open('$O/conv.jsonl'):
    d=json.loads(l); p=d['phases']
    print(d['tag'], d['prec'], d['step_ms'], ' '.join(f'{k}={p[k]:.4f}' for k in ('conv2_fwd','conv2_dgrad','conv2_wgrad','conv3_fwd','conv3_dgrad') if k in p))
"
SKIP_PROF=1 bash scripts/gpu_r4.sh ${1:-r4_v2}
