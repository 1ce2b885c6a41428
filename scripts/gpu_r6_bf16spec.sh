# Round 6: bf16 conv2 on the wave-specialised kernel (conv_ws_spec_kernel<EPI, 2, 1>) -- bf16 parity tests
# with the working tree, then the jingleback bf16 step A/B against HEAD's library (libabd_old.so)
mkdir -p gpurun_out/r6_bf16spec
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_bf16.py tests/test_gpu_conv_tiles.py > gpurun_out/r6_bf16spec/tests.txt 2>&1 || { tail -30 gpurun_out/r6_bf16spec/tests.txt; exit 1; }
tail -1 gpurun_out/r6_bf16spec/tests.txt
STEPS=100 BENCH_ARGS="--attack jingleback --gemm-precision bf16 --batch 256 --dropin-batches 0" bash scripts/lib_ab.sh r6_bf16spec old base
