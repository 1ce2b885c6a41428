#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/dbg3; mkdir -p $O
for prec in f32 f32split; do
  timeout -k 10 150 python scripts/share_debug.py $prec 2 20 >> $O/share.txt 2>&1 || { tail -20 $O/share.txt; exit 1; }
done
ABD_WS_DMA=0 timeout -k 10 150 python scripts/share_debug.py f32split 2 20 >> $O/share.txt 2>&1 || { tail -20 $O/share.txt; exit 1; }
grep "^(" $O/share.txt
