#!/bin/bash
# Wave-specialised conv kernel: parity tests, then an A/B against conv_ws_pre_kernel (libabd_nospec.so).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-spec1}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv_tiles.py tests/test_gpu_layers.py tests/test_gpu_smallcnn.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash scripts/gpu_ab.sh $T conv2_fwd,conv2_dgrad,conv3_fwd default nospec
