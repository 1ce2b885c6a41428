#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-dbg4}; mkdir -p $O
run() { echo "== $* $(date +%T)" >> $O/share.txt; timeout -k 10 170 "$@" >> $O/share.txt 2>&1 || { tail -20 $O/share.txt; exit 1; }; }
for i in 1 2 3 4 5 6 7 8; do ABD_LIB=$PWD/audio-backdoor-attack_amd/libabd_nopk.so ABD_WS_DMA=0 run python scripts/share_buffers.py f32split 2 60 32; done
echo "---- default build" >> $O/share.txt
for i in 1 2 3 4 5 6; do ABD_WS_DMA=0 run python scripts/share_buffers.py f32split 2 60 32; done
grep -v "^\[W\|amdgpu.ids" $O/share.txt | cut -c1-300
