#!/bin/bash
# Quick PMC (issue mix, MFMA busy, waits) + kernel trace over a short bench: bash scripts/pmc_kernels.sh TAG
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmck_${1:-x}
mkdir -p $O
B="python3 $R/bench.py --steps 3 --warmup 2 --profile-steps 1 --no-cpu"
timeout -s KILL 120 rocprofv3 --kernel-trace -d $O/kt -o kt -f csv -- $B > $O/kt.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES -d $O/b1 -o b1 -f csv -- $B > $O/b1.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE -d $O/b2 -o b2 -f csv -- $B > $O/b2.log 2>&1
echo "pmc rc $?"
