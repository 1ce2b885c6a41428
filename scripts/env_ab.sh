#!/bin/bash
# A/B of environment knobs on the headline bench (one GPU call): each VARIANT is "name:ENV=V,ENV2=V"
# (name "base" = no env); runs the list twice in order, prints ms/step and the per-phase times.
# Usage (on the box): bash scripts/env_ab.sh TAG "base" "pp8:ABD_HEAD_PP=8" ...
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
    env $envs timeout -k 10 240 python bench.py --steps ${STEPS:-100} --warmup 10 --no-cpu ${BENCH_ARGS:-} \
      > "$O/${name}_$rep.json" 2> "$O/${name}_$rep.err" || { tail -20 "$O/${name}_$rep.err"; exit 1; }
    python - "$O/${name}_$rep.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
ph = d.get("phases_ms_per_launch", {})
print(f"  ms/step {d['ms_per_step']:.4f}  value {d['value']:.0f}  " +
      " ".join(f"{k}={v*1000:.1f}" for k, v in ph.items() if k.startswith(("head", "conv2", "stft", "bn2"))))
PY
  done
done
