#!/bin/bash
# Run the GPU parity suite on the box; log under gpurun_out/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-run}
timeout -k 10 ${TEST_TIMEOUT:-900} python -m pytest tests -m gpu -q -rf -s ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?
echo "pytest exit $rc" >> gpurun_out/gpu_tests_$TAG.log
tail -80 gpurun_out/gpu_tests_$TAG.log
exit $rc
