set -u
cd $GRAFT_REPO_ROOT
out=gpurun_out/stftexp; mkdir -p $out
for rep in 1 2; do
for v in base g2n4 g2n3 g3n3 g2n2 g2n4b g2n4c g2n4d; do
  lib=audio-backdoor-attack_amd/libabd_$v.so; [ $v = base ] && lib=audio-backdoor-attack_amd/libabd.so
  echo "== $v"
  ABD_LIB=$PWD/$lib CFGS=n400,n2048 timeout -k 10 120 python scripts/stft_ab.py 100 || exit 1
done
done
