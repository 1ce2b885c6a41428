#!/bin/bash
# Copy one round_v3.sh run (gpurun_out/TAG) into the tracked profiles/: bench line, GPU test log,
# smoke, rocprofv3 kernel statistics, same-source HBM traffic per phase, per-config lines and the
# 2-rank gloo rehearsal.   Usage (here, after the gpurun call): bash scripts/collect_round.sh TAG
set -e
cd "$(dirname "$0")/.."
T=$1
O=gpurun_out/$T
P=profiles/$T
cp "$O/bench.json" "${P}_bench.json"
cp "$O/gpu_tests.log" "${P}_gpu_tests.txt"
cp "$O/smoke.log" "${P}_smoke.txt"
cp "$O/kt/kt_kernel_stats.csv" "${P}_kernel_stats.csv"
[ -f "$O/configs.jsonl" ] && cp "$O/configs.jsonl" "${P}_configs.jsonl"
[ -f "$O/bench_dp2_gloo.json" ] && cp "$O/bench_dp2_gloo.json" "${P}_bench_dp2_gloo_rehearsal.json"
if [ -d "$O/p_sq" ]; then mkdir -p "${P}_sq_pmc" && cp "$O"/p_sq/*counter_collection.csv "$O"/p_sq/*agent_info.csv "${P}_sq_pmc/"; fi
python scripts/traffic_json.py "$O" "${P}_traffic.json"
echo "collected $T"
