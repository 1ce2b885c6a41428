#!/bin/bash
# split-GEMM parity tests, then interleaved A/B benches of the f32split conv2 tile shapes (and f32).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_smallcnn.py tests/test_gpu_bf16.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_split_tests.log 2>&1 || { tail -30 gpurun_out/ab_split_tests.log; exit 1; }
tail -2 gpurun_out/ab_split_tests.log
bash scripts/ab_split_bench.sh
