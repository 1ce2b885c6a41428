#!/bin/bash
# Pre-split conv kernel: conv tile / layer / bf16 parity tests, then A/B against the DMA kernel
# (forward, ABD_WS_DMA=1; data gradient too, ABD_WS_DMA=2).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-pre1}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv_tiles.py tests/test_gpu_layers.py -q -x --timeout 240 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -5 $O/tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert" $O/tests.log | head -20; exit 1; }
for m in 1 2; do
  ABD_WS_DMA=$m bash scripts/gpu_ab.sh $1/m$m conv2_fwd,conv2_dgrad,conv2_wgrad default dma || exit 1
done
