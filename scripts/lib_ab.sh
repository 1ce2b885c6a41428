#!/bin/bash
# A/B of prebuilt library variants (audio-backdoor-attack_amd/libabd_<v>.so, scripts/build_variant.sh)
# on the headline bench, after the given parity tests pass with each variant.
# Usage (on the box): PYTEST_FILES="..." bash scripts/lib_ab.sh TAG base v1 v2 ...   ("base" = libabd.so)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/$1
shift
mkdir -p "$O"
set -o pipefail
lib() { [ "$1" = base ] && echo "$PWD/audio-backdoor-attack_amd/libabd.so" || echo "$PWD/audio-backdoor-attack_amd/libabd_$1.so"; }
if [ -n "${PYTEST_FILES:-}" ]; then
  for v in "$@"; do
    echo "== tests $v $(date +%T)"
    ABD_LIB=$(lib $v) timeout -k 10 400 python -u -m pytest ${PYTEST_FILES} -m gpu -x -q --timeout 200 --timeout-method thread \
      > "$O/tests_$v.log" 2>&1 || { tail -30 "$O/tests_$v.log"; exit 1; }
    tail -1 "$O/tests_$v.log"
  done
fi
for rep in 1 2; do
  for v in "$@"; do
    echo "== bench $v rep $rep $(date +%T)"
    ABD_LIB=$(lib $v) timeout -k 10 240 python bench.py --steps ${STEPS:-100} --warmup 10 --no-cpu ${BENCH_ARGS:-} \
      > "$O/${v}_$rep.json" 2> "$O/${v}_$rep.err" || { tail -20 "$O/${v}_$rep.err"; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); ph=d['phases_ms_per_launch']; print('  ms/step', d['ms_per_step'], {k: round(v*1000,1) for k,v in ph.items()})" "$O/${v}_$rep.json"
  done
done
