#!/bin/bash
# GPU: full parity suite + 2-rank DP rehearsal (gloo on one GPU) of the overlapped all-reduce step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-dp}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$TAG.txt 2>&1 || { tail -40 gpurun_out/gpu_tests_$TAG.txt; exit 1; }
tail -3 gpurun_out/gpu_tests_$TAG.txt
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 10 --warmup 3 --dist-backend gloo --no-cpu > gpurun_out/bench2_$TAG.json 2> gpurun_out/bench2_$TAG.err || { tail -30 gpurun_out/bench2_$TAG.err; exit 1; }
cut -c1-400 gpurun_out/bench2_$TAG.json
