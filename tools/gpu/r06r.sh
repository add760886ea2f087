#!/bin/bash
# r06r: GLV on / off for 2^22 and 2^24 BN254 MSMs (the default turns it off above 2^21)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
for rep in 1 2; do
  for g in 0 1; do
    timeout -k 10 200 python3 tools/msm_only.py --logn 24 --reps 5 --glv $g | tee -a gpurun_out/r06r.txt || exit 1
    timeout -k 10 200 python3 tools/msm_only.py --logn 22 --reps 5 --glv $g | tee -a gpurun_out/r06r.txt || exit 1
    timeout -k 10 300 python3 tools/msm_only.py --g2 --logn 22 --reps 3 --glv $g | tee -a gpurun_out/r06r.txt || exit 1
  done
done
for g in 0 1; do
  timeout -k 10 400 python3 tools/msm_only.py --g2 --logn 24 --reps 2 --glv $g | tee -a gpurun_out/r06r.txt || exit 1
done
