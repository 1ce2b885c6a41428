#!/bin/bash
# rocprofv3 kernel-trace + stats of a short bench run (no PMC counters here).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r}
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o bench --output-format csv \
  -- python3 bench.py --steps ${PROF_STEPS:-10} --warmup 3 --no-cpu > gpurun_out/prof_bench_$TAG.json 2> gpurun_out/prof_$TAG.err
rc=$?
find gpurun_out/prof_$TAG -name "*stats*" | head
cat gpurun_out/prof_bench_$TAG.json
exit $rc
