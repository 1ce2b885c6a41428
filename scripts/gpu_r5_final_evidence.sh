cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out/r5fin
timeout -k 10 900 python -u -m pytest -v -s --timeout 600 --timeout-method thread -m gpu tests/test_gpu_convergence.py --durations=0 > gpurun_out/r5fin/convergence.txt 2>&1 || { tail -30 gpurun_out/r5fin/convergence.txt; exit 1; }
grep -E "passed|failed" gpurun_out/r5fin/convergence.txt | tail -1
bash scripts/gpu_dp2_rehearsal.sh r5fin_dp2
