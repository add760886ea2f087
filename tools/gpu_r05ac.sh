#!/bin/bash
# r05ac (experiment): NTT DIF pass capped at four waves (alt build -DNTT_DIF_WPE=4, 34 VGPRs spilled) vs default.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05ac; mkdir -p $O && export TMPDIR=/tmp
ALT=$PWD/gnark-icicle_amd/libgnark_mi355x_alt.so
for rep in 1 2 3; do
  for v in def alt; do
    if [ $v = alt ]; then export GNARK_MI355X_LIB=$ALT; else unset GNARK_MI355X_LIB; fi
    timeout -k 10 120 python3 tools/ntt_only.py --logn 24 --reps 10 | sed "s/^/$v /" | tee -a $O/ab.txt
    timeout -k 10 120 python3 tools/ntt_only.py --logn 24 --reps 10 --coset | sed "s/^/$v /" | tee -a $O/ab.txt
  done
done
