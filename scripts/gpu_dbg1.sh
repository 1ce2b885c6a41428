#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/dbg1
timeout -k 10 200 python scripts/dp_debug.py > gpurun_out/dbg1/dp_debug.txt 2>&1; rc=$?
cat gpurun_out/dbg1/dp_debug.txt | grep -v Warning | tail -12
[ $rc -eq 0 ] || exit $rc
H=32 W=13 B=96 PORT=29562 timeout -k 10 200 python scripts/dp_debug.py > gpurun_out/dbg1/dp_debug_fm.txt 2>&1 || exit 1
tail -6 gpurun_out/dbg1/dp_debug_fm.txt
bash scripts/gpu_convexp.sh dbg1
