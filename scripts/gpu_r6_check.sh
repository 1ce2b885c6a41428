#!/bin/bash
# Round 6 quick GPU check: bench contract tests (N=1 and the self-spawned 2-rank gloo run), the
# default bench, and a rocprofv3 kernel-stats pass.  Usage: bash scripts/gpu_r6_check.sh TAG [pytest -k expr]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); O=$R/gpurun_out/$1; mkdir -p $O
set -o pipefail
echo "== tests $(date +%T)"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread -k "${2:-bench_contract}" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
echo "== bench $(date +%T)"
timeout -k 10 300 python bench.py --steps 200 --warmup 20 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['phases_ms_per_launch'])"
[ "${SKIP_PROF:-0}" = 1 ] && exit 0
cd /tmp && export TMPDIR=/tmp
echo "== kt $(date +%T)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt -f csv -- python3 $R/bench.py --steps 60 --warmup 20 --profile-steps 1 --no-cpu --dropin-batches 0 > $O/kt.log 2>&1 || { tail -20 $O/kt.log; exit 1; }
echo "== done $(date +%T)"
