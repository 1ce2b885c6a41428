#!/bin/bash
# Round-2 GPU session: parity suite (per-test timeouts, verbose progress), smoke, bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r2}
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread \
    ${PYTEST_ARGS:-} > gpurun_out/gpu_tests_$TAG.txt 2>&1
rc=$?
echo "pytest exit $rc" >> gpurun_out/gpu_tests_$TAG.txt
tail -25 gpurun_out/gpu_tests_$TAG.txt
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.txt 2>&1 || { cat gpurun_out/smoke_$TAG.txt; exit 1; }
tail -2 gpurun_out/smoke_$TAG.txt
timeout -k 10 600 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -30 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
exit $rc
