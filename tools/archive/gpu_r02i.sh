#!/bin/bash
# Round-2 verification (tools/gpu_r02_final.sh) plus a G2 window check (c = 15 / 16 / 17).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_r02_final.sh r02i || exit 1
{
for c in 15 16 17; do
  timeout -k 10 100 python tools/msm_only.py --g2 --reps 3 --window $c || exit 1
done
timeout -k 10 100 python tools/msm_only.py --reps 5 || exit 1
} 2>&1 | tee gpurun_out/r02i_g2win.txt
