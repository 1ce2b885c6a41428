#!/bin/bash
# Round-2 profiling session (each GPU step under its own timeout, chained with &&):
#   1. rocprofv3 --kernel-trace --stats of the default bench command (kernel averages + trace for gaps)
#   2. PMC passes on the feature stage alone (scripts/stft_only.py, B = 512 ultrasonic): issue mix,
#      wave states, LDS conflicts, HBM bytes (FETCH_SIZE / WRITE_SIZE in separate passes)
#   3. PMC passes over a short bench run (conv GEMMs)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=${1:-r2}
O=$R/gpurun_out/prof_$TAG
mkdir -p $O
BENCH="python3 $R/bench.py --steps 60 --warmup 10 --no-cpu"
STFT="python3 $R/scripts/stft_only.py"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt -f csv -- $BENCH > $O/kt.log 2>&1 &&
echo "kt done" &&
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES -d $O/s1 -o s1 -f csv -- $STFT > $O/s1.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE -d $O/s2 -o s2 -f csv -- $STFT > $O/s2.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/s3 -o s3 -f csv -- $STFT > $O/s3.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $O/s4 -o s4 -f csv -- $STFT > $O/s4.log 2>&1 &&
echo "stft pmc done" &&
BENCHS="python3 $R/bench.py --steps 3 --warmup 2 --profile-steps 1 --no-cpu" &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES -d $O/b1 -o b1 -f csv -- $BENCHS > $O/b1.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE -d $O/b2 -o b2 -f csv -- $BENCHS > $O/b2.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/b3 -o b3 -f csv -- $BENCHS > $O/b3.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/b4 -o b4 -f csv -- $BENCHS > $O/b4.log 2>&1 &&
echo "bench pmc done"
