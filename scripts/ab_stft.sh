#!/bin/bash
# Feature-stage A/B: parity tests on the current libabd.so, then scripts/stft_ab.py on each variant
#   bash scripts/ab_stft.sh tagA tagB ...   (tag "base" = libabd.so, others libabd_<tag>.so)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_mfcc.py \
  tests/test_gpu_pipeline.py ${AB_TESTS:-} > gpurun_out/ab_stft_tests.txt 2>&1 || { tail -30 gpurun_out/ab_stft_tests.txt; exit 1; }
tail -2 gpurun_out/ab_stft_tests.txt
for round in 1 2; do
  for t in "$@"; do
    lib=audio-backdoor-attack_amd/libabd.so; [ "$t" = base ] || lib=audio-backdoor-attack_amd/libabd_$t.so
    echo "== $t round $round"
    ABD_LIB=$PWD/$lib timeout -k 10 120 python3 -u scripts/stft_ab.py 50 || exit 1
  done
done
