#!/bin/bash
# Parity of the opt-in split kernels (ABD_WGRAD_SPLIT=1 weight gradient, ABD_HALO=1 halo conv)
# through the f32split GPU tests, then interleaved A/B benches.  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ABD_WGRAD_SPLIT=1 ABD_HALO=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_smallcnn.py tests/test_gpu_bf16.py -m gpu -x -q \
  -k f32split --timeout 120 --timeout-method thread > gpurun_out/ab_optin_tests.log 2>&1 || { tail -30 gpurun_out/ab_optin_tests.log; exit 1; }
tail -1 gpurun_out/ab_optin_tests.log
VARIANTS="${VARIANTS:-base:f32split:X=0 wgsplit:f32split:ABD_WGRAD_SPLIT=1}" KEYS=${KEYS:-conv2_fwd,conv2_dgrad,conv2_wgrad,conv3_wgrad} bash scripts/ab_split_bench.sh
