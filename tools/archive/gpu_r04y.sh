#!/bin/bash
# r04y: three MSMs in flight (gm_ctx::MSM_SLOTS = 3): async MSM parity, then the
# bench loop pipelined 2 vs 3 deep (GM_BENCH_PIPE_DEPTH), same box, and a trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-r04y}
GPU_MAX_HW_QUEUES=8 timeout -k 10 600 python -u -m pytest tests/test_msm_gpu.py -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for rep in 1 2 3; do
  for d in 2 3; do
    GM_BENCH_PIPE_DEPTH=$d timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-secondary --steps 20 --warmup 3 > gpurun_out/${T}_d$d.json 2> gpurun_out/${T}_d$d.err || { tail -20 gpurun_out/${T}_d$d.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/${T}_d$d.json')); print('depth=$d', d['value'], d['ms_per_step'], d['kernel_avg_ms']['msm_accum_g1'])" | tee -a gpurun_out/${T}_ab.txt
  done
done
GM_BENCH_PIPE_DEPTH=3 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_kt -o kt -- python3 bench.py --no-cpu-baseline --no-secondary --steps 20 --warmup 3 > /dev/null 2> gpurun_out/${T}_kt.err || { tail -30 gpurun_out/${T}_kt.err; exit 1; }
F=$(ls gpurun_out/${T}_kt/*kernel_trace.csv gpurun_out/${T}_kt/*/*kernel_trace.csv 2>/dev/null | head -1)
python3 tools/msm_timeline.py $F 16 > gpurun_out/${T}_msm_timeline.txt && head -45 gpurun_out/${T}_msm_timeline.txt
find gpurun_out/${T}_kt -name "*.csv" -size +5M -delete
