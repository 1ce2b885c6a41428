#!/bin/bash
# Sweep conv wgrad chunk rows (ABD_WGRAD_R2 / R3) with short bench runs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in ${R2S:-2 3 4 6}; do
  ABD_WGRAD_R2=$r timeout -k 10 120 python bench.py --steps 20 --no-cpu > gpurun_out/sweep_r2_$r.json 2>/dev/null || exit 1
  python3 -c "import json,sys; d=json.load(open('gpurun_out/sweep_r2_$r.json')); print('R2=$r', d['value'], d['phases_ms_per_launch']['conv2_wgrad'])"
done
for r in ${R3S:-4 8 12}; do
  ABD_WGRAD_R3=$r timeout -k 10 120 python bench.py --steps 20 --no-cpu > gpurun_out/sweep_r3_$r.json 2>/dev/null || exit 1
  python3 -c "import json,sys; d=json.load(open('gpurun_out/sweep_r3_$r.json')); print('R3=$r', d['value'], d['phases_ms_per_launch']['conv3_wgrad'])"
done
