#!/bin/bash
# Reduction A/B: segment length L (GM_MSM_SEGL) 2 vs 4 with the 512-thread bitsum, plus MSM parity tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_msm_gpu.py > gpurun_out/segl_tests.log 2>&1 || { tail -30 gpurun_out/segl_tests.log; exit 1; }
tail -2 gpurun_out/segl_tests.log
{
for L in 2 4 1; do
  export GM_MSM_SEGL=$L
  echo "L=$L"
  timeout -k 10 100 python tools/msm_only.py --reps 5 || exit 1
  timeout -k 10 100 python tools/msm_only.py --g2 --reps 3 || exit 1
  timeout -k 10 200 python tools/msm_only.py --curve bls12377 --g2 --logn 20 --reps 2 || exit 1
done
} 2>&1 | tee gpurun_out/segl.txt
