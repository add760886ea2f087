#!/bin/bash
# r05ad: Groth16 2^24 plain device-input proves, computeH queued after the wire plan (default) vs at once
# (GM_G16_H_AFTER_PLAN=0), re-measured with the r05 sort passes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05ad; mkdir -p $O && export TMPDIR=/tmp
for rep in 1 2 3; do
  for v in 1 0; do
    echo "== after_plan=$v rep $rep" >> $O/ab.txt
    GM_G16_H_AFTER_PLAN=$v timeout -k 10 300 python3 tools/g16_host_trace.py devonly >> $O/ab.txt 2>> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  done
done
grep -v "^mode" $O/ab.txt
