#!/bin/bash
# Round 6: the self-spawned multi-rank bench rehearsed on one GPU (gloo: RCCL refuses two ranks on one
# device), 2 and 4 ranks, then every config's step (bench_configs.py).  Usage: bash scripts/gpu_r6_multi.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/$1; mkdir -p $O
set -o pipefail
for n in 2 4; do
  echo "== gloo dp$n $(date +%T)"
  timeout -k 10 300 python bench.py --gpus $n --dist-backend gloo --steps 20 --warmup 5 --no-cpu --dropin-batches 0 \
    --n-train 2048 > $O/bench_gloo_dp$n.json 2> $O/bench_gloo_dp$n.err || { tail -20 $O/bench_gloo_dp$n.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_gloo_dp$n.json')); print(d['n_gpus'], d['config']['parallelism'], d['value'], d['ms_per_step'], d['train_metrics'])"
done
echo "== configs $(date +%T)"
timeout -k 10 600 python scripts/bench_configs.py --steps 50 > $O/configs.jsonl 2> $O/configs.err || { tail -20 $O/configs.err; exit 1; }
cat $O/configs.jsonl | cut -c1-220
