#!/bin/bash
# Accumulation tuning sweep: slice size (GM_MSM_SLICE) and the G2 kernel variant
# (GM_MSM_ACCUM), on the bench MSM lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for sl in 32 64 128; do
  GM_MSM_SLICE=$sl timeout -k 10 120 python bench.py --no-cpu-baseline --no-secondary --steps 20 > gpurun_out/sw_$sl.json || exit 1
  python3 -c "
import json; d=json.load(open('gpurun_out/sw_$sl.json')); print('slice $sl', d['ms_per_step'], d['kernel_avg_ms']['msm_accum_g1'])"
done
for v in noprefetch prefetch; do
  GM_MSM_ACCUM=$v timeout -k 10 120 python tools/tune_window.py --cases bn254:g2:20 --reps 5 --span 0 > gpurun_out/g2_$v.txt || exit 1
  echo "g2 accum $v"; tail -1 gpurun_out/g2_$v.txt
done
