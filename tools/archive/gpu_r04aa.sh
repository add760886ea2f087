#!/bin/bash
# r04aa: bench loop 3 deep with 8 vs 16 hardware queues (does every slot stream get a
# queue of its own at 8?), same box, plus a trace at 16.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-r04aa}
for rep in 1 2 3; do
  for q in 8 16; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-secondary --steps 20 --warmup 3 > gpurun_out/${T}_q$q.json 2> gpurun_out/${T}_q$q.err || { tail -20 gpurun_out/${T}_q$q.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/${T}_q$q.json')); print('q=$q', d['value'], d['ms_per_step'], d['kernel_avg_ms']['msm_accum_g1'])" | tee -a gpurun_out/${T}_ab.txt
  done
done
GPU_MAX_HW_QUEUES=16 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_kt -o kt -- python3 bench.py --no-cpu-baseline --no-secondary --steps 20 --warmup 3 > /dev/null 2> gpurun_out/${T}_kt.err || { tail -30 gpurun_out/${T}_kt.err; exit 1; }
F=$(ls gpurun_out/${T}_kt/*kernel_trace.csv gpurun_out/${T}_kt/*/*kernel_trace.csv 2>/dev/null | head -1)
python3 tools/msm_timeline.py $F 16 > gpurun_out/${T}_msm_timeline.txt && head -45 gpurun_out/${T}_msm_timeline.txt
find gpurun_out/${T}_kt -name "*.csv" -size +5M -delete
