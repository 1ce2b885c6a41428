#!/bin/bash
# Second pass of scripts/gpu_pk_opsel.sh with more launches: V=0 / V=1 / V=2 as two probe
# processes beside one train-step process, then V=0 as ONE probe process alone on the GPU.
set -u
out=gpurun_out/pkopsel2
mkdir -p $out
for V in 0 1 2 0 1 2; do
  echo "== V=$V: two probe processes beside one train-step process $(date +%T)"
  timeout -k 10 200 python scripts/share_buffers.py f32split 1 1500 32 > $out/nb_$V.txt 2>&1 & nb=$!
  timeout -k 10 200 ./scripts/pk_opsel_probe $V 3000 & a=$!
  timeout -k 10 200 ./scripts/pk_opsel_probe $V 3000 & b=$!
  wait $a; ra=$?; wait $b; rb=$?; wait $nb; rn=$?
  grep -v amdgpu.ids $out/nb_$V.txt | tail -1
  echo "rc $ra $rb $rn"
  if [ $ra -ne 0 ] || [ $rb -ne 0 ] || [ $rn -ne 0 ]; then exit 1; fi
done
echo "== V=0: one probe process alone $(date +%T)"
timeout -k 10 200 ./scripts/pk_opsel_probe 0 6000 || exit 1
