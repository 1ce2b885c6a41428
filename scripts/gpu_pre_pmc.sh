#!/bin/bash
# SQ counters of the pre-split conv kernel (default build) vs the DMA kernel (libabd_dma.so).
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/${1:-prepmc}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
CMD="python3 $R/bench.py --steps 3 --warmup 2 --profile-steps 1 --no-cpu --dropin-batches 0"
for v in default dma; do
  L=$R/audio-backdoor-attack_amd/libabd.so; [ $v != default ] && L=$R/audio-backdoor-attack_amd/libabd_$v.so
  ABD_WS_DMA=2 ABD_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES -d $O/$v -o p -f csv -- $CMD > $O/$v.log 2>&1 || { tail -5 $O/$v.log; exit 1; }
done
for v in default dma; do for k in conv_ws_pre_kernel conv_ws_dma_kernel conv_ws_split_kernel; do
  python3 $R/scripts/pmc_summary.py $O/$v "$k<" 2>/dev/null | grep -E "INSTS|WAVE_CYCLES|WAIT_ANY|MFMA_BUSY|SQ_WAVES" | sed "s/^/$v $k /"
done; done
