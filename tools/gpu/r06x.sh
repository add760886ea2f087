#!/bin/bash
# r06x: kernel traces (after r06t / r06v) of 2^24 device-input proves (plain, precomputed) for the exposed-time analysis
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
for V in plain precomputed; do
  A=""; [ $V = precomputed ] && A="--precompute"
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r06x_kt_$V -o kt -- python3 tools/g16_only.py --logn 24 --reps 1 $A > gpurun_out/r06x_$V.out 2>&1 || { tail -5 gpurun_out/r06x_$V.out; exit 1; }
  TR=$(find gpurun_out/r06x_kt_$V -name "*kernel_trace.csv" | head -1)
  python3 tools/g16_exposed.py "$TR" | tee gpurun_out/r06x_exposed_$V.txt
  gzip -f "$TR"
done
