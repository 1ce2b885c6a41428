#!/bin/bash
# PMC passes over a short bench run for the train-step kernels (conv GEMMs, pools, head): issue /
# wait mix, MFMA busy and the vector-memory pipeline (TA / TD / L1).  One GPU call.
# Usage (on the box): bash scripts/pmc_conv_r3.sh TAG
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$1
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
CMD="python3 $R/bench.py --steps 3 --warmup 2 --profile-steps 1 --no-cpu"
p() { echo "== $1 $(date +%T)"; n=$1; shift; timeout -s KILL 120 rocprofv3 --pmc "$@" -d "$O/$n" -o p -f csv -- $CMD > "$O/$n.log" 2>&1 || { tail -5 "$O/$n.log"; exit 1; }; }
p sq1 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR
p sq2 SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE
p tx TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum GRBM_GUI_ACTIVE
echo "== done $(date +%T)"
