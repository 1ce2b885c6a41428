#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/dbg2
timeout -k 10 200 python scripts/dp_debug.py > gpurun_out/dbg2/dp_debug.txt 2>&1; rc=$?
grep -v "Warning\|socket\|Gloo\|amdgpu.ids" gpurun_out/dbg2/dp_debug.txt | tail -12
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python scripts/dp_overlap_debug.py f32 f32split > gpurun_out/dbg2/overlap.txt 2>&1; rc=$?
grep -v "Warning\|socket\|Gloo\|amdgpu.ids" gpurun_out/dbg2/overlap.txt | tail -20
exit $rc
