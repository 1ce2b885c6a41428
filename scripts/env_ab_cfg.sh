#!/bin/bash
# A/B of environment knobs on one bench configuration: BENCH_ARGS selects it (e.g. "--attack flowmur
# --batch 256 --gemm-precision bf16"); each VARIANT is "name:ENV=V,ENV2=V" ("base" = no env).
# Usage (on the box): BENCH_ARGS="..." bash scripts/env_ab_cfg.sh TAG "base" "x:ABD_X=1" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/$1
shift
mkdir -p "$O"
set -o pipefail
for rep in 1 2; do
  for v in "$@"; do
    name=${v%%:*}
    envs=""
    [ "$v" != "$name" ] && envs=$(echo "${v#*:}" | tr ',' ' ')
    echo "== $name rep $rep ($envs) $(date +%T)"
    env $envs timeout -k 10 240 python bench.py --steps ${STEPS:-200} --warmup 20 --no-cpu ${BENCH_ARGS:-} \
      > "$O/${name}_$rep.json" 2> "$O/${name}_$rep.err" || { tail -20 "$O/${name}_$rep.err"; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print('  ms/step', d['ms_per_step'], {k: round(v*1000,1) for k,v in d.get('phases_ms_per_launch',{}).items() if k.startswith(('conv','head','bn'))})" "$O/${name}_$rep.json"
  done
done
