#!/bin/bash
# bf16 plane-operand GEMMs on the register-prefetch kernel (default) vs conv_ws_dma_kernel
# (libabd_padma.so): bf16 parity, then jingleback / flowmur bf16 benches alternated.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-pareg}
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bf16.py \
  tests/test_gpu_conv_tiles.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for cfg in "jingleback 256" "flowmur 256"; do
  set -- $cfg
  STEPS=100 BENCH_ARGS="--dropin-batches 0 --attack $1 --batch $2 --gemm-precision bf16" bash scripts/lib_ab.sh $(basename $O)_$1 base padma || exit 1
done
