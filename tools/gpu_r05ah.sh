#!/bin/bash
# r05ah (experiment): BLS12-377 G1 accumulation variants -- prefetching group kernel (default), with one mad chain
# per product (GM_MSM_PF_CHAIN=1, 209 VGPRs), chain without prefetch at three waves (=3, 168 VGPRs).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05ah; mkdir -p $O && export TMPDIR=/tmp
for v in 1 3; do
  GM_MSM_PF_CHAIN=$v timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_msm_gpu.py -k "bls12377 and not g2" > $O/tests_$v.log 2>&1 || { tail -30 $O/tests_$v.log; exit 1; }
  tail -1 $O/tests_$v.log
done
for rep in 1 2 3; do
  for v in 0 1 3; do
    GM_MSM_PF_CHAIN=$v timeout -k 10 120 python3 tools/msm_only.py --curve bls12377 --logn 22 --reps 5 | sed "s/^/pf_chain=$v /" | tee -a $O/ab.txt
  done
done
