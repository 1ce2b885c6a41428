#!/bin/bash
# PMC passes on the feature stage alone (scripts/stft_only.py, B = 512 ultrasonic), one pass per run:
#   bash scripts/pmc_stft.sh TAG   -> gpurun_out/pmc_TAG/{s1,s2,s3,s4}
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_${1:-x}
mkdir -p $O
STFT="python3 $R/scripts/stft_only.py"
timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $O/kt -o kt -f csv -- $STFT > $O/kt.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES -d $O/s1 -o s1 -f csv -- $STFT > $O/s1.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE -d $O/s2 -o s2 -f csv -- $STFT > $O/s2.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_IFETCH SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_MISC -d $O/s5 -o s5 -f csv -- $STFT > $O/s5.log 2>&1
echo "pmc rc $?"
