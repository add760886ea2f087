#!/bin/bash
# r04ad: with three MSMs in flight the bucket reduction overlaps the next
# accumulation -- does the window optimum move (2^20 GLV: c = 16 -> 8 windows;
# 19 -> 7 windows, 8x the buckets)?  Also the accumulation slice length.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-r04ad}
for rep in 1 2; do
  for v in "W=0" "W=17" "W=18" "W=19" "S=32" "S=128"; do
    case $v in W=*) E="GM_BENCH_MSM_WINDOW=${v#W=}" ;; S=*) E="GM_MSM_SLICE=${v#S=}" ;; esac
    env $E timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-secondary > gpurun_out/${T}.json 2> gpurun_out/${T}.err || { tail -20 gpurun_out/${T}.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/${T}.json')); print('$v', d['value'], d['ms_per_step'], d['kernel_avg_ms'])" | tee -a gpurun_out/${T}_sweep.txt
  done
done
