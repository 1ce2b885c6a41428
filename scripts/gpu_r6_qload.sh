# Round 6: STFT queue stealing with counter loads -- feature-stage A/B (HEAD library as libabd_old.so vs
# the working tree) at B = 512 and 256, then the MFCC GPU tests
mkdir -p gpurun_out/r6_qload
for bb in 512 256; do
  for v in _old "" _old "" _old ""; do echo "B $bb lib$v"; B=$bb ABD_LIB=$PWD/audio-backdoor-attack_amd/libabd$v.so timeout -k 10 120 python scripts/feature_phase_time.py || exit 1; done
done > gpurun_out/r6_qload/ab.txt 2>&1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_mfcc_scale.py tests/test_gpu_mfcc.py tests/test_gpu_flowmur.py tests/test_gpu_daba.py > gpurun_out/r6_qload/tests.txt 2>&1
