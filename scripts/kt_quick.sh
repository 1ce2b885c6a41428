#!/bin/bash
# Kernel trace + stats of a short bench: [BENCH_ARGS=...] bash scripts/kt_quick.sh TAG [ENV=VAL ...]  -> gpurun_out/ktq_TAG
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=${1:-x}; shift
O=$R/gpurun_out/ktq_$T
mkdir -p $O
for e in "$@"; do export "$e"; done
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O -o kt -f csv -- python3 $R/bench.py --steps 20 --warmup 5 --profile-steps 1 --no-cpu --dropin-batches 0 $BENCH_ARGS > $O/kt.log 2>&1
echo "kt rc $?"
