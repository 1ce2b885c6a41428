#!/bin/bash
# bf16 vs f32split bench lines for BASELINE configs[2] (jingleback, B = 256) and configs[4]
# (flowmur, B = 256), plus rocprofv3 kernel statistics of the bf16 runs.  One GPU call.
# Usage (on the box): bash scripts/prof_bf16.sh TAG
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
O=$R/gpurun_out/$1
mkdir -p "$O"
set -o pipefail
step() { echo "== $1 $(date +%T)"; }
# alternating order, twice: box clock / warm-up drift shows as a rep-to-rep difference, not as a
# precision difference
for rep in 1 2; do
for A in jingleback flowmur; do
  for P in f32split bf16; do
    step "bench $A $P rep $rep"
    timeout -k 10 300 python bench.py --attack $A --batch 256 --gemm-precision $P --steps 200 --warmup 20 --no-cpu \
      > "$O/bench_${A}_${P}_$rep.json" 2> "$O/bench_${A}_${P}_$rep.err" || { tail -20 "$O/bench_${A}_${P}_$rep.err"; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['ms_per_step'], d['value'])" "$O/bench_${A}_${P}_$rep.json"
  done
done
done
cd /tmp && export TMPDIR=/tmp
for A in jingleback flowmur; do
  step "kernel-trace $A bf16"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/kt_$A" -o kt -f csv -- \
    python3 $R/bench.py --attack $A --batch 256 --gemm-precision bf16 --steps 10 --warmup 3 --profile-steps 1 --no-cpu \
    > "$O/kt_$A.log" 2>&1 || { tail -20 "$O/kt_$A.log"; exit 1; }
done
step done
