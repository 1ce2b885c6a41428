#!/bin/bash
# Round-4 evidence on the final code: PMC passes (conv GEMMs, STFT), per-config bench lines, and
# rocprofv3 kernel statistics for jingleback / flowmur at B = 256 in bf16 and f32split.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-r4_p1}
O=gpurun_out/$T; mkdir -p $O
bash scripts/pmc_r4.sh $T/pmc || exit 1
timeout -k 10 400 python scripts/bench_configs.py --steps 20 > $O/configs.jsonl 2> $O/configs.err || { tail -20 $O/configs.err; exit 1; }
cut -c1-200 $O/configs.jsonl
for cfg in "jingleback bf16" "jingleback f32split" "flowmur bf16" "flowmur f32split"; do
  set -- $cfg
  bash scripts/prof_config.sh $T/${1}_$2 $1 $2 256 || exit 1
done
echo "== done $(date +%T)"
