#!/bin/bash
# Feature-stage ablations (ABD_STFT_ABLATE bits: 1 skip sample loads, 2 skip FFTs, 4 skip power/mel)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for a in 0 1 2 4 6 7; do
  echo "== ablate $a"
  ABD_STFT_ABLATE=$a timeout -k 10 120 python3 -u scripts/stft_ab.py 50 2>&1 | grep ultra || exit 1
done
