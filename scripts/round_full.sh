#!/bin/bash
# One GPU call: parity suite -> smoke -> bench -> rocprofv3 kernel stats -> FETCH/WRITE PMC passes.
# Every GPU step has its own time limit; the script stops at the first failure.
# Usage (on the box): bash scripts/round_full.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
O=$R/gpurun_out/$1
mkdir -p "$O"
python scripts/traffic_json.py --print-sha > "$O/csrc_sha1.txt"
set -o pipefail
step() { echo "== $1 $(date +%T)"; }

if [ "${SKIP_TESTS:-0}" != 1 ]; then
  step tests
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread \
    ${PYTEST_K:+-k "$PYTEST_K"} > "$O/gpu_tests.log" 2>&1 || { tail -40 "$O/gpu_tests.log"; exit 1; }
  tail -3 "$O/gpu_tests.log"
  step smoke
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { tail -30 "$O/smoke.log"; exit 1; }
  tail -1 "$O/smoke.log"
fi
step bench
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > "$O/bench.json" 2> "$O/bench.err" || { tail -30 "$O/bench.err"; exit 1; }
cat "$O/bench.json"
[ "${SKIP_PROF:-0}" = 1 ] && exit 0
cd /tmp && export TMPDIR=/tmp
CMD="python3 $R/bench.py --steps 10 --warmup 3 --profile-steps 1 --no-cpu --dropin-batches 0"
step kernel-trace
# 60 steps after 20 warmup: the per-kernel averages are steady-state launches, comparable with the
# bench line's live brackets (10 steps averaged in the cold first launches: stft_mel +10 %)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/kt" -o kt -f csv -- \
  python3 $R/bench.py --steps 60 --warmup 20 --profile-steps 1 --no-cpu --dropin-batches 0 > "$O/kt.log" 2>&1 || { tail -20 "$O/kt.log"; exit 1; }
[ "${SKIP_PMC:-0}" = 1 ] && exit 0
step pmc-fetch
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d "$O/p_fetch" -o p -f csv -- $CMD > "$O/p_fetch.log" 2>&1 || { tail -20 "$O/p_fetch.log"; exit 1; }
step pmc-write
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d "$O/p_write" -o p -f csv -- $CMD > "$O/p_write.log" 2>&1 || { tail -20 "$O/p_write.log"; exit 1; }
if [ "${SQ_PMC:-1}" = 1 ]; then
  step pmc-sq
  timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
    -d "$O/p_sq" -o p -f csv -- $CMD > "$O/p_sq.log" 2>&1 || { tail -20 "$O/p_sq.log"; exit 1; }
fi
step done
