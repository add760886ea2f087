#!/bin/bash
# Run the primary bench line R times on one box (run-to-run spread of ms_per_step).
#   bash tools/bench_repeat.sh [R]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
R=${1:-3}
for i in $(seq 1 "$R"); do
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-secondary --steps 20 > gpurun_out/rep_$i.json 2> gpurun_out/rep_$i.err || { tail -20 gpurun_out/rep_$i.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/rep_$i.json')); print(d['ms_per_step'], d['kernel_avg_ms'])"
done
