#!/bin/bash
# SQ / TA / TCP counters of the conv2 GEMM kernels: default build (conv_ws_spec_kernel) against
# libabd_nospec.so (conv_ws_pre_kernel).  Usage (on the box): bash scripts/pmc_spec.sh TAG
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$1
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
BENCH="python3 $R/bench.py --steps 3 --warmup 2 --profile-steps 1 --no-cpu --dropin-batches 0"
p() {
  local n=$1 lib=$2; shift 2
  echo "== $n $(date +%T)"
  ABD_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc "$@" -d "$O/$n" -o p -f csv -- $BENCH > "$O/$n.log" 2>&1 || { tail -5 "$O/$n.log"; exit 1; }
}
for v in default nospec; do
  L=$R/audio-backdoor-attack_amd/libabd.so; [ $v != default ] && L=$R/audio-backdoor-attack_amd/libabd_$v.so
  p ${v}_sq1 $L SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR
  p ${v}_sq2 $L SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE
  p ${v}_tx $L TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum GRBM_GUI_ACTIVE
done
for v in default nospec; do for k in "conv_ws_spec_kernel<1, 2>" "conv_ws_pre_kernel<1, 2>" "conv_ws_spec_kernel<0, 2>" "conv_ws_pre_kernel<0, 2>"; do
  for pp in sq1 sq2 tx; do python3 $R/scripts/pmc_summary.py $O/${v}_$pp "$k" 2>/dev/null | sed "s/^/$v $pp $k | /"; done
done; done > $O/summary.txt
echo "== done $(date +%T)"
