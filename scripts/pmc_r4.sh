#!/bin/bash
# Round-4 PMC passes (one GPU call): the train-step kernels of bench.py (issue / wait mix, MFMA busy,
# LDS conflicts, vector-memory pipeline, HBM bytes via TCC_EA0 FETCH / WRITE in passes of their own)
# and the Bluestein STFT alone (scripts/stft_only.py: wait fraction, LDS FIFO pressure).
# Every pass is its own rocprofv3 run under a hard kill; counters per block stay within the
# single-pass limits (<= 8 SQ, <= 4 TCC, <= 4 TCP, <= 2 TA, <= 2 TD, <= 2 GRBM).
# Usage (on the box): bash scripts/pmc_r4.sh TAG
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$1
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
BENCH="python3 $R/bench.py --steps 3 --warmup 2 --profile-steps 1 --no-cpu --dropin-batches 0"
STFT="python3 $R/scripts/stft_only.py"
p() {
  local n=$1 cmd=$2; shift 2
  echo "== $n $(date +%T)"
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d "$O/$n" -o p -f csv -- $cmd > "$O/$n.log" 2>&1 || { tail -5 "$O/$n.log"; exit 1; }
}
p conv_sq1 "$BENCH" SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR
p conv_sq2 "$BENCH" SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE
p conv_tx "$BENCH" TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum GRBM_GUI_ACTIVE
p conv_fetch "$BENCH" FETCH_SIZE
p conv_write "$BENCH" WRITE_SIZE
p stft_sq1 "$STFT" SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD
p stft_sq2 "$STFT" SQ_INST_LEVEL_VMEM SQ_INST_CYCLES_VMEM_RD SQ_THREAD_CYCLES_VALU SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE
p stft_sq3 "$STFT" SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR
echo "== done $(date +%T)"
