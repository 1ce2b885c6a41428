#!/bin/bash
# Round-4 GPU call: parity suite (all failures listed, not -x), smoke, bench, rocprofv3 kernel stats.
# Test FAILURES (pytest exit 1) do not stop the call; a timeout, abort or crash of any step does.
#   bash scripts/gpu_r4.sh TAG      (PYTEST_K / SKIP_TESTS / SKIP_PROF / BENCH_ARGS as in round_full.sh)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
O=$R/gpurun_out/$1
mkdir -p "$O"
python scripts/traffic_json.py --print-sha > "$O/csrc_sha1.txt"
step() { echo "== $1 $(date +%T)"; }
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  step tests
  timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread \
    ${PYTEST_K:+-k "$PYTEST_K"} > "$O/gpu_tests.log" 2>&1
  rc=$?
  tail -25 "$O/gpu_tests.log"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "pytest exit $rc: stopping"; exit $rc; }
  step smoke
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { tail -30 "$O/smoke.log"; exit 1; }
  tail -1 "$O/smoke.log"
fi
step bench
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > "$O/bench.json" 2> "$O/bench.err" || { tail -30 "$O/bench.err"; exit 1; }
cut -c1-1500 "$O/bench.json"
[ "${SKIP_PROF:-0}" = 1 ] && exit 0
cd /tmp && export TMPDIR=/tmp
CMD="python3 $R/bench.py --steps 10 --warmup 3 --profile-steps 1 --no-cpu --dropin-batches 0 ${BENCH_ARGS:-}"
step kernel-trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/kt" -o kt -f csv -- $CMD > "$O/kt.log" 2>&1 || { tail -20 "$O/kt.log"; exit 1; }
step done
