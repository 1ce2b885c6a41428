#!/bin/bash
# Build libabd_<tag>.so with extra compile flags for mfcc.hip only (STFT plan A/B experiments),
# linked with the default objects of the other sources (run `make` first).  Select with ABD_LIB=...
set -e
cd "$(dirname "$0")/../audio-backdoor-attack_amd"
TAG=$1; shift
mkdir -p build_$TAG
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function \
  -Xclang -target-feature -Xclang -packed-fp32-ops -fno-signed-zeros "$@" -c csrc/mfcc.hip -o build_$TAG/mfcc.hip.o \
  2>&1 | grep -v "not a recognized feature" || true
objs=$(ls build/*.o | grep -v mfcc.hip.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o libabd_$TAG.so $objs build_$TAG/mfcc.hip.o
