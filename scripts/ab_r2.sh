#!/bin/bash
# A/B of library variants on the feature stage and the bench: bash scripts/ab_r2.sh tagA tagB ...
# (tag "base" = libabd.so; others = libabd_<tag>.so from scripts/build_variant.sh)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for round in 1 2; do
  for t in "$@"; do
    lib=audio-backdoor-attack_amd/libabd.so; [ "$t" = base ] || lib=audio-backdoor-attack_amd/libabd_$t.so
    echo "== $t round $round"
    ABD_LIB=$PWD/$lib timeout -k 10 120 python3 -u scripts/stft_ab.py 50 || exit 1
    ABD_LIB=$PWD/$lib timeout -k 10 180 python3 -u bench.py --steps 200 --warmup 20 --no-cpu --profile-steps 2 > gpurun_out/ab_${t}_$round.json || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/ab_${t}_$round.json'));print('bench', d['ms_per_step'], d['value'], d['phases_ms_per_launch']['stft_mel'])"
  done
done
