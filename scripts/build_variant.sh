#!/bin/bash
# Build libabd_<tag>.so with extra compile flags (A/B experiments; select with ABD_LIB=...).
set -e
cd "$(dirname "$0")/../audio-backdoor-attack_amd"
TAG=$1; shift
mkdir -p build_$TAG
for f in capi.cpp prof.cpp mfcc.hip smallcnn.hip daba.hip resample.hip effects.hip; do
  extra=""; [ $f = mfcc.hip ] && extra="-fno-signed-zeros"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Xclang -target-feature -Xclang -packed-fp32-ops $extra "$@" -c csrc/$f -o build_$TAG/$f.o 2>&1 | grep -v "not a recognized feature" &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o libabd_$TAG.so build_$TAG/*.o
