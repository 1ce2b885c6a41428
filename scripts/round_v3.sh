#!/bin/bash
# Round measurement: parity suite, smoke, bench, rocprofv3 stats + HBM PMC passes (round_full.sh),
# then the per-config bench and a 2-rank DP rehearsal (gloo on the one GPU).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r1_v3}
bash scripts/round_full.sh $TAG || exit 1
O=gpurun_out/$TAG
echo "== configs $(date +%T)"
timeout -k 10 400 python scripts/bench_configs.py --steps 20 > $O/configs.jsonl 2> $O/configs.err || { tail -20 $O/configs.err; exit 1; }
cat $O/configs.jsonl
echo "== dp2 $(date +%T)"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 10 --warmup 3 --dist-backend gloo --no-cpu > $O/bench_dp2_gloo.json 2> $O/bench_dp2_gloo.err || { tail -30 $O/bench_dp2_gloo.err; exit 1; }
cut -c1-300 $O/bench_dp2_gloo.json
echo "== done $(date +%T)"
