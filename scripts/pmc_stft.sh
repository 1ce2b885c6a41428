set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/pmc/kt -o kt -f csv -- python3 $R/scripts/stft_only.py > $R/gpurun_out/pmc/kt.log 2>&1
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES -d $R/gpurun_out/pmc/p1 -o p1 -f csv -- python3 $R/scripts/stft_only.py > $R/gpurun_out/pmc/p1.log 2>&1
timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INST_LEVEL_LDS -d $R/gpurun_out/pmc/p2 -o p2 -f csv -- python3 $R/scripts/stft_only.py > $R/gpurun_out/pmc/p2.log 2>&1
