#!/bin/bash
# One GPU call: selected GPU tests (PYTEST_K / files), then optional bench lines (BENCH_LINES="attack:prec:batch ...").
# Usage (on the box): PYTEST_FILES="tests/test_gpu_styles.py" bash scripts/gpu_quick.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/$1
mkdir -p "$O"
set -o pipefail
if [ -n "${PYTEST_FILES:-}" ]; then
  echo "== tests $(date +%T)"
  timeout -k 10 600 python -u -m pytest ${PYTEST_FILES} -m gpu -x -v --timeout 300 --timeout-method thread \
    ${PYTEST_K:+-k "$PYTEST_K"} > "$O/tests.log" 2>&1 || { tail -60 "$O/tests.log"; exit 1; }
  grep -E "PASSED|FAILED|passed|failed" "$O/tests.log" | tail -30
fi
for rep in 1 2; do
  for L in ${BENCH_LINES:-}; do
    IFS=: read -r A P B <<< "$L"
    echo "== bench $A $P $B rep $rep $(date +%T)"
    timeout -k 10 300 python bench.py --attack $A --batch $B --gemm-precision $P --steps ${STEPS:-200} --warmup 20 --no-cpu \
      > "$O/bench_${A}_${P}_${B}_$rep.json" 2> "$O/bench_${A}_${P}_${B}_$rep.err" || { tail -20 "$O/bench_${A}_${P}_${B}_$rep.err"; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['ms_per_step'], d['value'], {k: round(v*1000,1) for k,v in d.get('phases_ms_per_launch',{}).items()})" "$O/bench_${A}_${P}_${B}_$rep.json"
  done
done
echo "== done $(date +%T)"
