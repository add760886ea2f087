#!/bin/bash
# r04l: the bench's pipelined MSM loop with the two in-flight MSMs on their own
# streams (GM_MSM_SLOT_STREAMS=1) vs one stream, same box, then a kernel trace of
# the two-stream loop (does MSM i+1's conversion / sort overlap MSM i's reduction?).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-r04l}
for rep in 1 2 3; do
  for v in 0 1; do
    GM_MSM_SLOT_STREAMS=$v timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-secondary --steps 20 --warmup 3 > gpurun_out/${T}_b$v.json 2> gpurun_out/${T}_b$v.err || { tail -20 gpurun_out/${T}_b$v.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/${T}_b$v.json')); print('slot_streams=$v', d['value'], d['ms_per_step'], d['kernel_avg_ms']['msm_accum_g1'])" | tee -a gpurun_out/${T}_ab.txt
  done
done
GM_MSM_SLOT_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_kt -o kt -- python3 bench.py --no-cpu-baseline --no-secondary --steps 20 --warmup 3 > /dev/null 2> gpurun_out/${T}_kt.err || { tail -30 gpurun_out/${T}_kt.err; exit 1; }
F=$(ls gpurun_out/${T}_kt/*kernel_trace.csv gpurun_out/${T}_kt/*/*kernel_trace.csv 2>/dev/null | head -1)
python3 tools/msm_timeline.py $F 16 > gpurun_out/${T}_msm_timeline.txt && head -50 gpurun_out/${T}_msm_timeline.txt
find gpurun_out/${T}_kt -name "*.csv" -size +5M -delete
