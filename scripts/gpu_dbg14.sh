#!/bin/bash
# Packed-FP32 determinism with processes sharing the GPU (scripts/pk_probe.hip).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-dbg14}; mkdir -p $O
echo "== one process" >> $O/pk.txt
timeout -k 10 100 ./scripts/pk_probe 1500 >> $O/pk.txt 2>&1 || { cat $O/pk.txt; exit 1; }
for np in 2 4; do
  echo "== $np processes" >> $O/pk.txt
  pids=""
  for i in $(seq $np); do timeout -k 10 150 ./scripts/pk_probe 1500 >> $O/pk.txt 2>&1 & pids="$pids $!"; done
  for p in $pids; do wait $p || { echo "probe failed"; cat $O/pk.txt; exit 1; }; done
done
echo "== pk_probe beside two train-step processes" >> $O/pk.txt
ABD_WS_DMA=0 timeout -k 10 150 python scripts/share_buffers.py f32split 2 200 32 >> $O/pk.txt 2>&1 & p1=$!
sleep 10
timeout -k 10 120 ./scripts/pk_probe 1500 >> $O/pk.txt 2>&1 || { cat $O/pk.txt; exit 1; }
wait $p1 || { cat $O/pk.txt; exit 1; }
grep -v "^\[W\|amdgpu.ids" $O/pk.txt | cut -c1-300
