#!/bin/bash
# Round profile: rocprofv3 kernel stats of the default bench command, then HBM bytes per launch from
# separate FETCH_SIZE / WRITE_SIZE passes on a short bench (MI355X_MICROARCH.md HBM section).
#   bash scripts/prof_round.sh TAG   -> gpurun_out/prof_TAG/{kt,b3,b4}
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_${1:-x}
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt -f csv -- python3 $R/bench.py --steps 200 --warmup 20 --no-cpu > $O/kt.log 2>&1 &&
echo "kt done" &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/b3 -o b3 -f csv -- python3 $R/bench.py --steps 3 --warmup 2 --profile-steps 1 --no-cpu > $O/b3.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/b4 -o b4 -f csv -- python3 $R/bench.py --steps 3 --warmup 2 --profile-steps 1 --no-cpu > $O/b4.log 2>&1 &&
echo "traffic done"
