#!/bin/bash
# does packed-FP32 low-lane operand selection go wrong under GPU sharing?
# Each variant of scripts/pk_opsel_probe runs as two processes beside one train-step process (the
# round-4 reproducer's neighbour); then the round-4 reproducer itself on the packed library.
# scripts/libabd_pk.so = libabd built WITHOUT the Makefile's PKFLAGS (packed FP32 on), e.g.
#   for f in capi.cpp prof.cpp mfcc.hip smallcnn.hip daba.hip resample.hip effects.hip; do
#     hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC [-fno-signed-zeros for mfcc.hip] \
#       -c audio-backdoor-attack_amd/csrc/$f -o /tmp/pkbuild/$f.o; done
#   hipcc --offload-arch=gfx950 -shared -o scripts/libabd_pk.so /tmp/pkbuild/*.o
set -u
out=gpurun_out/pkopsel
mkdir -p $out
for V in 0 1 2; do
  echo "== V=$V: two probe processes beside one train-step process $(date +%T)"
  timeout -k 10 150 python scripts/share_buffers.py f32split 1 600 32 > $out/nb_$V.txt 2>&1 & nb=$!
  timeout -k 10 150 ./scripts/pk_opsel_probe $V 1500 & a=$!
  timeout -k 10 150 ./scripts/pk_opsel_probe $V 1500 & b=$!
  wait $a; ra=$?; wait $b; rb=$?; wait $nb; rn=$?
  grep -v amdgpu.ids $out/nb_$V.txt
  echo "rc $ra $rb $rn"
  if [ $ra -ne 0 ] || [ $rb -ne 0 ] || [ $rn -ne 0 ]; then exit 1; fi
done
for k in 1 2 3 4 5 6; do
  echo "== packed libabd, two train-step processes, run $k $(date +%T)"
  ABD_LIB=scripts/libabd_pk.so timeout -k 10 120 python scripts/share_buffers.py f32split 2 60 32 2>&1 | grep -v amdgpu.ids || exit 1
done
