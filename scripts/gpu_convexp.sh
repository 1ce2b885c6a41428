#!/bin/bash
# Conv2 GEMM diagnosis: MFMA issue-rate probe variants, then the train-step kernel times of the
# default build and the conv_ws_dma_kernel ablation builds (libabd_abl<bits>.so, -DABD_DMA_ABL).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-convexp}; mkdir -p $O
for v in 0 1 2 3 4; do timeout -k 5 60 ./scripts/mfma_probe $v 1000 >> $O/probe.txt 2>&1 || exit 1; done
cat $O/probe.txt
for lib in ${LIBS:-libabd.so libabd_abl1.so libabd_abl2.so libabd_abl4.so libabd_abl8.so}; do
  ABD_LIB=$PWD/audio-backdoor-attack_amd/$lib timeout -k 10 120 python scripts/conv_probe.py --tag $lib ${PROBE_ARGS:-} >> $O/conv.jsonl 2>> $O/conv.err || { tail -20 $O/conv.err; exit 1; }
done
ABD_LIB=$PWD/audio-backdoor-attack_amd/libabd.so timeout -k 10 120 python scripts/conv_probe.py --prec bf16 --tag bf16 >> $O/conv.jsonl 2>> $O/conv.err || exit 1
python3 -c "
import json,sys
for l in open('$O/conv.jsonl'):
    d=json.loads(l); p=d['phases']
    print(d['tag'], d['prec'], d['step_ms'], ' '.join(f'{k}={p[k]:.4f}' for k in ('conv2_fwd','conv2_dgrad','conv2_wgrad','conv3_fwd') if k in p))
"
