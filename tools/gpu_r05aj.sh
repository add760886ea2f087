#!/bin/bash
# r05aj (experiment): BN254 G2 lane-pair accumulation with one mad chain per product (GM_MSM_PAIR_CHAIN=1: prefetch, 2 waves,
# 179 VGPRs; =3 with GM_MSM_PAIR_PF=0: no prefetch, 3 waves, 168 VGPRs) vs default (prefetch, 2 waves, 200 VGPRs).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05aj; mkdir -p $O && export TMPDIR=/tmp
GM_MSM_PAIR_CHAIN=3 GM_MSM_PAIR_PF=0 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_msm_gpu.py -k "bn254 and (g2 or True)" > $O/tests3.log 2>&1 || { tail -30 $O/tests3.log; exit 1; }
tail -1 $O/tests3.log
GM_MSM_PAIR_CHAIN=1 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_msm_gpu.py -k "bn254" > $O/tests1.log 2>&1 || { tail -30 $O/tests1.log; exit 1; }
tail -1 $O/tests1.log
for rep in 1 2 3; do
  for v in "0 1" "1 1" "3 0"; do
    set -- $v
    GM_MSM_PAIR_CHAIN=$1 GM_MSM_PAIR_PF=$2 timeout -k 10 120 python3 tools/msm_only.py --g2 --logn 20 --reps 5 | sed "s/^/chain=$1 pf=$2 /" | tee -a $O/ab.txt
  done
done
for rep in 1 2; do
  for v in "0 1" "3 0"; do
    set -- $v
    echo "== g16 chain=$1 pf=$2" >> $O/ab.txt
    GM_MSM_PAIR_CHAIN=$1 GM_MSM_PAIR_PF=$2 timeout -k 10 300 python3 tools/g16_host_trace.py devonly >> $O/ab.txt 2>> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  done
done
grep -v "^mode" $O/ab.txt
