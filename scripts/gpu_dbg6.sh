#!/bin/bash
# LDS integrity with two processes sharing the GPU (scripts/lds_probe.hip), then one alone.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-dbg6}; mkdir -p $O
for kb in 128 32; do
  echo "== two processes, $kb KB" >> $O/lds.txt
  timeout -k 10 120 ./scripts/lds_probe $kb 20 20000 >> $O/lds.txt 2>&1 & p1=$!
  timeout -k 10 120 ./scripts/lds_probe $kb 20 20000 >> $O/lds.txt 2>&1 & p2=$!
  wait $p1 || { echo "probe 1 failed"; cat $O/lds.txt; exit 1; }
  wait $p2 || { echo "probe 2 failed"; cat $O/lds.txt; exit 1; }
done
echo "== one process, 128 KB" >> $O/lds.txt
timeout -k 10 120 ./scripts/lds_probe 128 20 20000 >> $O/lds.txt 2>&1 || { cat $O/lds.txt; exit 1; }
echo "== four processes, 128 KB" >> $O/lds.txt
pids=""
for i in 1 2 3 4; do timeout -k 10 150 ./scripts/lds_probe 128 10 20000 >> $O/lds.txt 2>&1 & pids="$pids $!"; done
for p in $pids; do wait $p || { echo "probe failed"; cat $O/lds.txt; exit 1; }; done
cat $O/lds.txt
