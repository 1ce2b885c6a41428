#!/bin/bash
# r4_v3: sharing-determinism probe, conv probes (bf16 plane DMA, ABD_WS_DMA 0/1/2), parity suite, bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r4_v3}; mkdir -p $O
for prec in f32 f32split; do
  timeout -k 10 150 python scripts/share_debug.py $prec 2 20 >> $O/share.txt 2>&1 || { tail -20 $O/share.txt; exit 1; }
done
ABD_WS_DMA=0 timeout -k 10 150 python scripts/share_debug.py f32split 2 20 >> $O/share.txt 2>&1 || { tail -20 $O/share.txt; exit 1; }
grep "^(" $O/share.txt
for prec in bf16 f32split; do for m in 0 1 2; do
  ABD_WS_DMA=$m timeout -k 10 120 python scripts/conv_probe.py --prec $prec --tag dma$m >> $O/conv.jsonl 2>> $O/conv.err || { tail -20 $O/conv.err; exit 1; }
done; done
python3 -c "
import json
for l in open('$O/conv.jsonl'):
    d=json.loads(l); p=d['phases']
    print(d['tag'], d['prec'], d['step_ms'], ' '.join(f'{k}={p[k]:.4f}' for k in ('conv2_fwd','conv2_dgrad','conv2_wgrad','conv3_fwd','conv3_dgrad') if k in p))
"
SKIP_PROF=1 bash scripts/gpu_r4.sh ${1:-r4_v3}
