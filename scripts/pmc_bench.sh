#!/bin/bash
# rocprofv3 kernel-trace + PMC passes over a short bench run (one counter group per pass).
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmcb
mkdir -p $O
CMD="python3 $R/bench.py --steps 3 --warmup 2 --profile-steps 1 --no-cpu"
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/kt -o kt -f csv -- $CMD > $O/kt.log 2>&1
timeout -k 10 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES -d $O/p1 -o p1 -f csv -- $CMD > $O/p1.log 2>&1
timeout -k 10 180 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA -d $O/p2 -o p2 -f csv -- $CMD > $O/p2.log 2>&1
timeout -k 10 180 rocprofv3 --pmc FETCH_SIZE -d $O/p3 -o p3 -f csv -- $CMD > $O/p3.log 2>&1
timeout -k 10 180 rocprofv3 --pmc WRITE_SIZE -d $O/p4 -o p4 -f csv -- $CMD > $O/p4.log 2>&1
