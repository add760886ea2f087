#!/bin/bash
# r03q: window-size sweep (msm_only --window) around the cost-model choice for the
# bench / config MSMs, two alternated repetitions.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-r03q}
for rep in 1 2; do
  for c in 16 17 18; do
    for args in "--curve bls12377 --g2 --logn 22 --reps 2" "--curve bls12377 --logn 22 --reps 3"; do
      timeout -k 10 200 python tools/msm_only.py $args --window $c || exit 1
    done
  done
  for c in 15 16 17; do
    for args in "--logn 20 --reps 10" "--g2 --logn 20 --reps 4"; do
      timeout -k 10 200 python tools/msm_only.py $args --window $c || exit 1
    done
  done
done > gpurun_out/${T}_sweep.txt 2>&1 || { tail -20 gpurun_out/${T}_sweep.txt; exit 1; }
cut -c1-120 gpurun_out/${T}_sweep.txt
