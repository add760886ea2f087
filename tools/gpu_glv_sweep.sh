#!/bin/bash
# Slice length (GM_MSM_SLICE) and reduction segment length (GM_MSM_SEGL) sweep of
# the GLV 2^20 BN254 G1 bench line, same box, 2 runs each.
#   bash tools/gpu_glv_sweep.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${1:-glvsw}
out=gpurun_out/${T}.txt
: > $out
run() {
  for rep in 1 2; do
    r=$(env "$@" timeout -k 10 120 python bench.py --no-cpu-baseline --no-secondary --steps 20 2>/dev/null | tail -1) || { echo "fail $*" >> $out; exit 1; }
    echo "$* rep$rep $(echo "$r" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["kernel_avg_ms"])')" >> $out
  done
}
run GM_MSM_SLICE=64
run GM_MSM_SLICE=32
run GM_MSM_SLICE=128
run GM_MSM_SEGL=2
run GM_MSM_SEGL=8
run GM_MSM_SEGL=16
cat $out
