#!/bin/bash
# Sort radix-width sweep on the bench MSM (GM_SORT_BITS), then MSM parity tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for b in 0 8 11; do
  GM_SORT_BITS=$b timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary > gpurun_out/sort_$b.json || exit 1
  python3 -c "
import json; d=json.load(open('gpurun_out/sort_$b.json')); print('bits $b', d['ms_per_step'], d['kernel_avg_ms'])"
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "msm or groth16" > gpurun_out/sort_tests.log 2>&1 || { tail -30 gpurun_out/sort_tests.log; exit 1; }
tail -2 gpurun_out/sort_tests.log
