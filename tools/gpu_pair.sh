#!/bin/bash
# G2 lane pairs (accumulation, fixup, reduction): MSM parity tests, then pair vs one-lane A/B (GM_MSM_ACCUM).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_msm_gpu.py > gpurun_out/pair_tests.log 2>&1 || { tail -30 gpurun_out/pair_tests.log; exit 1; }
tail -2 gpurun_out/pair_tests.log
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_configs_full.py -k "bls12377" > gpurun_out/pair_tests_bls.log 2>&1 || { tail -30 gpurun_out/pair_tests_bls.log; exit 1; }
tail -2 gpurun_out/pair_tests_bls.log
{
for A in pair noprefetch; do
  export GM_MSM_ACCUM=$A
  echo "accum=$A"
  timeout -k 10 100 python tools/msm_only.py --g2 --reps 3 || exit 1
  timeout -k 10 100 python tools/msm_only.py --g2 --reps 3 --precompute || exit 1
  timeout -k 10 200 python tools/msm_only.py --curve bls12377 --g2 --logn 22 --reps 2 || exit 1
done
} 2>&1 | tee gpurun_out/pair.txt
