#!/bin/bash
# Interleaved A/B benches: VARIANTS="name:precision:ENV=..,ENV2=.. ..." (2 rounds each).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do
  for v in ${VARIANTS:-mi1:f32split:ABD_SPLIT_MI=1 mi2:f32split:ABD_SPLIT_MI=2 f32:f32:X=0}; do
    name=${v%%:*}; rest=${v#*:}; prec=${rest%%:*}; envs=${rest#*:}
    env $(echo "$envs" | tr ',' ' ') timeout -k 10 120 python bench.py --steps 30 --no-cpu --gemm-precision $prec > gpurun_out/ab_${name}_$r.json 2>gpurun_out/ab_${name}_$r.err || { tail -20 gpurun_out/ab_${name}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/ab_${name}_$r.json')); p=d['phases_ms_per_launch']; print('$name', $r, d['value'], d['ms_per_step'], ' '.join(f'{k}={p[k]:.4f}' for k in '${KEYS:-conv2_fwd,conv2_dgrad,conv2_wgrad,conv3_fwd,conv3_dgrad}'.split(',')))"
  done
done
