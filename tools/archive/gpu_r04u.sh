#!/bin/bash
# r04u: which prior use makes the 2^24 host-input prove fast (r04r: 204 -> 171 ms
# after staged proves)?  Fresh process per mode.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
for m in fresh stage async device; do
  timeout -k 10 300 python3 -u tools/g16_host_trace.py $m 2>&1 | grep -E "mode|prove" | tee -a gpurun_out/r04u.txt || exit 1
done
