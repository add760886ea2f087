#!/bin/bash
# r06ab: window size sweep of the 2^24 G2 and G1 MSMs (plain points, uniform scalars; default c = 20)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
for w in 0 18 19 21; do
  timeout -k 10 300 python3 tools/msm_only.py --g2 --logn 24 --reps 2 --window $w | tee -a gpurun_out/r06ab.txt || exit 1
done
for w in 0 19 21; do
  timeout -k 10 300 python3 tools/msm_only.py --logn 24 --reps 3 --window $w | tee -a gpurun_out/r06ab.txt || exit 1
done
