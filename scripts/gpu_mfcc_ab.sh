#!/bin/bash
# mfcc.hip change vs the previous one (libabd_prev.so): feature parity (every frame at B = 512,
# ragged DABA rows, FlowMur, the persistent grid capped), the feature stage alone, the headline bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-mfab}
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_mfcc.py \
  tests/test_gpu_mfcc_scale.py tests/test_gpu_daba.py tests/test_gpu_flowmur.py tests/test_gpu_pipeline.py \
  > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for rep in 1 2; do
  for v in base prev; do
    L=$PWD/audio-backdoor-attack_amd/libabd.so; [ $v = prev ] && L=$PWD/audio-backdoor-attack_amd/libabd_prev.so
    echo "== stft $v rep $rep"
    ABD_LIB=$L timeout -k 10 120 python scripts/stft_ab.py 100 || exit 1
  done
done
STEPS=100 BENCH_ARGS="--dropin-batches 0" bash scripts/lib_ab.sh $(basename $O)_ab base prev
