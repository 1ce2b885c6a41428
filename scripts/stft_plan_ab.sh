set -u
cd $GRAFT_REPO_ROOT
out=gpurun_out/stftexp; mkdir -p $out
for rep in 1 2; do
for v in base f2048pp2 f2048pp1 f400pp8 f400pp6 f400r20pp12 f400r20pp6 f400pp13n3 f400pp17; do
  lib=audio-backdoor-attack_amd/libabd_$v.so; [ $v = base ] && lib=audio-backdoor-attack_amd/libabd.so
  echo "== $v"
  ABD_LIB=$PWD/$lib CFGS=n400,n2048 timeout -k 10 120 python scripts/stft_ab.py 100 || exit 1
done
done
