#!/bin/bash
# r04j: kernel trace of the default bench MSM loop (pipelined gm_msm_async, two slots):
# how much of each step the accumulation covers and what overlaps it.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-r04j}
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_kt -o kt -- python3 bench.py --no-cpu-baseline --no-secondary --steps 20 --warmup 3 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_kt.err || { tail -30 gpurun_out/${T}_kt.err; exit 1; }
F=$(ls gpurun_out/${T}_kt/*kernel_trace.csv gpurun_out/${T}_kt/*/*kernel_trace.csv 2>/dev/null | head -1)
python3 tools/msm_timeline.py $F 16 > gpurun_out/${T}_msm_timeline.txt && head -60 gpurun_out/${T}_msm_timeline.txt
