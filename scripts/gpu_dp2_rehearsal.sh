#!/bin/bash
# The bench's N > 1 path rehearsed on the one-GPU box: two ranks on GPU 0 over gloo (RCCL cannot
# host two ranks on one device), launched the way the driver launches N > 1.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-dp2}
mkdir -p $O
export MASTER_ADDR=127.0.0.1 HIP_VISIBLE_DEVICES=0
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29561 bench.py --gpus 2 --steps 20 --warmup 5 --dist-backend gloo --no-cpu \
  > $O/bench_dp2_gloo.json 2> $O/bench_dp2_gloo.err || { tail -30 $O/bench_dp2_gloo.err; exit 1; }
tail -1 $O/bench_dp2_gloo.json | cut -c1-400
