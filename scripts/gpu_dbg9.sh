#!/bin/bash
# Cross-process detector: the LDS probe (pattern-checked LDS in every block) runs beside a train-step
# loop; mismatches in the probe mean some train-step kernel wrote outside its own LDS, and
# differences in the train step beside a probe that only touches its own LDS mean preemption /
# sharing alone perturbs the step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-dbg9}; mkdir -p $O
for kb in 32 64 128; do
  echo "== step loop beside lds_probe $kb KB" >> $O/x.txt
  ABD_WS_DMA=0 timeout -k 10 170 python scripts/share_buffers.py f32split 1 150 32 >> $O/x.txt 2>&1 & p1=$!
  sleep 8
  timeout -k 10 120 ./scripts/lds_probe $kb 40 20000 >> $O/x.txt 2>&1 & p2=$!
  wait $p2 || { echo "probe failed"; cat $O/x.txt; exit 1; }
  wait $p1 || { echo "step loop failed"; cat $O/x.txt; exit 1; }
done
grep -v "^\[W\|amdgpu.ids" $O/x.txt | cut -c1-700
