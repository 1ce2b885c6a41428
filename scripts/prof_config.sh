#!/bin/bash
# rocprofv3 kernel statistics + bench line for one non-headline workload (e.g. jingleback bf16).
# Usage (on the box): bash scripts/prof_config.sh TAG ATTACK PRECISION BATCH
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); O=$R/gpurun_out/$1; mkdir -p $O
ARGS="--attack $2 --gemm-precision $3 --batch $4 --no-cpu"
timeout -k 10 300 python bench.py $ARGS > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-400 $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt -f csv -- python3 $R/bench.py $ARGS --steps 10 --warmup 3 --profile-steps 1 > $O/kt.log 2>&1 || { tail -20 $O/kt.log; exit 1; }
echo done
