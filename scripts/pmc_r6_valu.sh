#!/bin/bash
# Round 6: dynamic VALU instruction mix (fp32 add / mul / fma / transcendental, int32, int64, cvt) of
# the Bluestein STFT alone (scripts/stft_only.py) and of the train-step kernels (bench.py), one
# rocprofv3 pass each under a hard kill (8 SQ counters per pass).
# Usage (on the box): bash scripts/pmc_r6_valu.sh TAG; summary: scripts/pmc_r4_summary.py RUN OUT
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$1
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
BENCH="python3 $R/bench.py --steps 3 --warmup 2 --profile-steps 1 --no-cpu --dropin-batches 0"
STFT="python3 $R/scripts/stft_only.py"
MIX="SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT"
p() {
  local n=$1 cmd=$2; shift 2
  echo "== $n $(date +%T)"
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d "$O/$n" -o p -f csv -- $cmd > "$O/$n.log" 2>&1 || { tail -5 "$O/$n.log"; exit 1; }
}
p stft_mix "$STFT" $MIX
p conv_mix "$BENCH" $MIX
echo "== done $(date +%T)"
