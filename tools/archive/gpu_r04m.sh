#!/bin/bash
# r04m: do the bench's two in-flight MSMs overlap once their slot streams get HW
# queues of their own?  GPU_MAX_HW_QUEUES=8 (HIP's default 4 is shared by torch's,
# the context's stream / aux / copy streams and both slot streams) with
# GM_MSM_SLOT_STREAMS=1, against the default; then a kernel trace of the former.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-r04m}
for rep in 1 2 3; do
  for v in base q8slot q8; do
    case $v in
      base) E="" ;;
      q8slot) E="GPU_MAX_HW_QUEUES=8 GM_MSM_SLOT_STREAMS=1" ;;
      q8) E="GPU_MAX_HW_QUEUES=8" ;;
    esac
    env $E timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-secondary --steps 20 --warmup 3 > gpurun_out/${T}_$v.json 2> gpurun_out/${T}_$v.err || { tail -20 gpurun_out/${T}_$v.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/${T}_$v.json')); print('$v', d['value'], d['ms_per_step'], d['kernel_avg_ms']['msm_accum_g1'])" | tee -a gpurun_out/${T}_ab.txt
  done
done
export GPU_MAX_HW_QUEUES=8 GM_MSM_SLOT_STREAMS=1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_kt -o kt -- python3 bench.py --no-cpu-baseline --no-secondary --steps 20 --warmup 3 > /dev/null 2> gpurun_out/${T}_kt.err || { tail -30 gpurun_out/${T}_kt.err; exit 1; }
F=$(ls gpurun_out/${T}_kt/*kernel_trace.csv gpurun_out/${T}_kt/*/*kernel_trace.csv 2>/dev/null | head -1)
python3 tools/msm_timeline.py $F 16 > gpurun_out/${T}_msm_timeline.txt && head -50 gpurun_out/${T}_msm_timeline.txt
find gpurun_out/${T}_kt -name "*.csv" -size +5M -delete
