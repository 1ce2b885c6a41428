#!/bin/bash
# Per-table-row SNR scales (abd_inject.row_scale): parity of the feature stage and the FlowMur
# pipeline / convergence tests, then the FlowMur bench against the previous library.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-rsc}
mkdir -p $O
[ "${SKIP_TESTS:-0}" = 1 ] || timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_mfcc_scale.py \
  tests/test_gpu_mfcc.py tests/test_gpu_flowmur.py tests/test_gpu_pipeline.py tests/test_gpu_flowmur_dp.py tests/test_gpu_ops.py \
  > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
[ "${SKIP_TESTS:-0}" = 1 ] || tail -1 $O/tests.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 500 --timeout-method thread -m gpu tests/test_gpu_convergence.py -k flowmur \
  > $O/conv.txt 2>&1 || { tail -30 $O/conv.txt; exit 1; }
tail -1 $O/conv.txt
STEPS=100 BENCH_ARGS="--dropin-batches 0 --attack flowmur --batch 256" bash scripts/lib_ab.sh $(basename $O)_ab base prev
