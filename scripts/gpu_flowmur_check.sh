#!/bin/bash
# FlowMur / injection parity after the row_scale change, then the FlowMur bench and its kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-fmchk}
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_flowmur.py \
  tests/test_gpu_mfcc.py tests/test_gpu_mfcc_scale.py tests/test_gpu_pipeline.py tests/test_gpu_flowmur_dp.py \
  > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for a in flowmur; do
  timeout -k 10 240 python bench.py --attack $a --batch 256 --steps 100 --warmup 10 --no-cpu --dropin-batches 0 > $O/bench_$a.json 2> $O/bench_$a.err || exit 1
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d['phases_ms_per_launch'].get('row_scale'))" $O/bench_$a.json $a
done
BENCH_ARGS="--attack flowmur --batch 256" bash scripts/kt_quick.sh fm_$(basename $O)
