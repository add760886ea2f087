#!/bin/bash
# Window-size sweep with the current library: per-kernel times per c.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
{
for w in 14 15 16; do timeout -k 10 100 python tools/msm_only.py --window $w --reps 5 || exit 1; done
for w in 14 15 16; do timeout -k 10 100 python tools/msm_only.py --g2 --window $w --reps 3 || exit 1; done
for w in 15 16 17; do timeout -k 10 200 python tools/msm_only.py --curve bls12377 --logn 22 --window $w --reps 2 || exit 1; done
for w in 15 16 17; do timeout -k 10 300 python tools/msm_only.py --curve bls12377 --g2 --logn 22 --window $w --reps 1 || exit 1; done
} 2>&1 | tee gpurun_out/win_sweep.txt
