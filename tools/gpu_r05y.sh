#!/bin/bash
# r05y (experiment): Groth16 2^24 device-input proves vs the prove's MSM streams
# (GM_G16_MSM_STREAMS 0/1/2, GM_G16_MSM_PRIO 0/1), then the Groth16 GPU tests with 2 / prio.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05y; mkdir -p $O && export TMPDIR=/tmp
for rep in 1 2; do
  for v in "0 0" "1 0" "2 0" "1 1" "2 1"; do
    set -- $v
    echo "== streams=$1 prio=$2 rep $rep" >> $O/ab.txt
    GM_G16_MSM_STREAMS=$1 GM_G16_MSM_PRIO=$2 timeout -k 10 300 python3 tools/g16_host_trace.py devonly >> $O/ab.txt 2>> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  done
done
GM_G16_MSM_STREAMS=2 GM_G16_MSM_PRIO=1 timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_groth16_gpu.py tests/test_r1cs_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
grep -v "^mode" $O/ab.txt
