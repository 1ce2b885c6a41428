#!/bin/bash
# Round-5 check on the GPU: the layer / conv / BN parity tests, the convergence
# suite, then the headline bench.  Every step has its own time limit; stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r5chk}
mkdir -p $O
echo "== parity $(date +%T)"
timeout -k 10 500 python -u -m pytest -x -q --timeout 250 --timeout-method thread -m gpu tests/test_gpu_layers.py \
  tests/test_gpu_smallcnn.py tests/test_gpu_bn_gamma.py tests/test_gpu_conv_tiles.py tests/test_gpu_guards.py \
  > $O/parity.txt 2>&1 || { tail -30 $O/parity.txt; exit 1; }
tail -2 $O/parity.txt
echo "== convergence $(date +%T)"
timeout -k 10 900 python -u -m pytest -v -s --timeout 600 --timeout-method thread -m gpu tests/test_gpu_convergence.py \
  --durations=0 > $O/convergence.txt 2>&1 || { grep -E "PASSED|FAILED|Error|assert" $O/convergence.txt | tail -30; exit 1; }
grep -E "passed|failed" $O/convergence.txt | tail -2
echo "== bench $(date +%T)"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json;d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['roofline']['frac'])"
