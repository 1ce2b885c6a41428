#!/bin/bash
# PMC passes over the feature stage alone (scripts/stft_only.py): issue / wait mix, vector-memory
# pipeline (TA / TD / L1) and LDS FIFO pressure of the Bluestein STFT kernel.  One GPU call.
# Usage (on the box): bash scripts/pmc_stft_r3.sh TAG
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$1
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
CMD="python3 $R/scripts/stft_only.py"
p() { echo "== $1 $(date +%T)"; shift_name=$1; shift; timeout -s KILL 90 rocprofv3 --pmc "$@" -d "$O/$shift_name" -o p -f csv -- $CMD > "$O/$shift_name.log" 2>&1 || { tail -5 "$O/$shift_name.log"; exit 1; }; }
p sq1 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD
p sq2 SQ_INST_LEVEL_VMEM SQ_INST_CYCLES_VMEM_RD SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_THREAD_CYCLES_VALU SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE
p tx TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum GRBM_GUI_ACTIVE
p sq3 SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAVES
echo "== done $(date +%T)"
