#!/bin/bash
# Scalar-FP32 build: GPU-sharing determinism probe, then the parity suite, smoke, bench, kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r4_v5}; mkdir -p $O
for m in 0 1 0 1; do
  ABD_WS_DMA=$m timeout -k 10 170 python scripts/share_buffers.py f32split 2 60 32 >> $O/share.txt 2>&1 || { tail -20 $O/share.txt; exit 1; }
done
grep "^(" $O/share.txt | cut -c1-200
bash scripts/gpu_r4.sh ${1:-r4_v5}
