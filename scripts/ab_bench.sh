#!/bin/bash
# A/B bench on one box: VARIANTS="NAME:ENV=..,ENV2=.. NAME2:..." ; ROUNDS interleaved runs each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-3}); do
  for v in $VARIANTS; do
    name=${v%%:*}; envs=${v#*:}
    envargs=$(echo "$envs" | tr ',' ' ')
    env $envargs timeout -k 10 120 python bench.py --steps ${STEPS:-30} --no-cpu > gpurun_out/ab_${name}_$r.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/ab_${name}_$r.json')); p=d['phases_ms_per_launch']; print('$name', $r, d['value'], ' '.join(f'{k}={p[k]:.4f}' for k in '${KEYS:-stft_mel}'.split(',')))"
  done
done
