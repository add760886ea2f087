#!/bin/bash
# r04t: fresh-process 2^24 host-input proves: copy stream at normal vs highest
# priority (GM_COPY_STREAM_PRIO), with 8 and 4 hardware queues.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-r04t}
for q in 8 4; do
  for p in 0 1; do
    echo "GPU_MAX_HW_QUEUES=$q GM_COPY_STREAM_PRIO=$p" | tee -a gpurun_out/${T}.txt
    GPU_MAX_HW_QUEUES=$q GM_COPY_STREAM_PRIO=$p timeout -k 10 300 python3 -u tools/g16_host_trace.py 2>&1 | grep prove | tee -a gpurun_out/${T}.txt || exit 1
  done
done
