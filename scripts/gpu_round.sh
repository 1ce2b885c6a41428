#!/bin/bash
# GPU session: parity tests, smoke, bench, rocprof kernel stats.  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r}
set -o pipefail
timeout -k 10 900 python -m pytest tests -m gpu -q -rf > gpurun_out/gpu_tests_$TAG.log 2>&1; rc=$?
echo "pytest exit $rc" >> gpurun_out/gpu_tests_$TAG.log; tail -15 gpurun_out/gpu_tests_$TAG.log
[ $rc -eq 0 ] || [ "${CONTINUE_ON_FAIL:-0}" = 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { cat gpurun_out/smoke_$TAG.log; exit 1; }
tail -2 gpurun_out/smoke_$TAG.log
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -30 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
