#!/bin/bash
# Env-knob A/B on the headline bench: bash scripts/ab_env.sh "NAME=VAL ..." "NAME=VAL ..." ...
#   ("base" = no extra env).  Runs AB_TESTS first (parity), then 2 rounds of bench.py per setting.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -n "${AB_TESTS:-}" ]; then
  timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread $AB_TESTS \
    > gpurun_out/ab_env_tests.txt 2>&1 || { tail -30 gpurun_out/ab_env_tests.txt; exit 1; }
  tail -2 gpurun_out/ab_env_tests.txt
fi
for round in 1 2; do
  i=0
  for e in "$@"; do
    i=$((i+1))
    envs=""; [ "$e" = base ] || envs="$e"
    env $envs timeout -k 10 180 python3 -u bench.py --steps 200 --warmup 20 --no-cpu --profile-steps 2 \
      > gpurun_out/ab_env_${i}_$round.json 2> gpurun_out/ab_env_${i}_$round.err || { tail -20 gpurun_out/ab_env_${i}_$round.err; exit 1; }
    python3 -c "
import json,sys;d=json.load(open('gpurun_out/ab_env_${i}_$round.json'));p=d['phases_ms_per_launch']
print('%-32s %.4f ms/step %8.0f utt/s | stft %.4f dct %.4f c2f %.4f c2d %.4f c2w %.4f' % ('$e', d['ms_per_step'], d['value'], p.get('stft_mel',0), p.get('db_dct',0), p.get('conv2_fwd',0), p.get('conv2_dgrad',0), p.get('conv2_wgrad',0)))"
  done
done
