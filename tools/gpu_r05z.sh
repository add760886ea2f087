#!/bin/bash
# r05z (experiment): Groth16 Z MSM queued before K on its own stream (GM_G16_Z_FIRST=1; =2: K waits
# for Z's plan), 2^24 device-input and host-input proves, plain key; Groth16 tests with the variant.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05z; mkdir -p $O && export TMPDIR=/tmp
GM_G16_Z_FIRST=2 timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_groth16_gpu.py tests/test_r1cs_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  for v in 0 1 2; do
    echo "== z_first=$v rep $rep" >> $O/ab.txt
    GM_G16_Z_FIRST=$v timeout -k 10 300 python3 tools/g16_host_trace.py devonly >> $O/ab.txt 2>> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  done
done
GM_G16_Z_FIRST=2 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o tr -- python3 tools/g16_host_trace.py devonly > /dev/null 2> $O/trace.err || { tail -30 $O/trace.err; exit 1; }
python3 tools/g16_timeline.py $(ls $O/tr/*kernel_trace.csv $O/tr/*/*kernel_trace.csv 2>/dev/null | head -1) --all > $O/timeline_all.txt || exit 1
find $O/tr -name "*.csv" -delete
grep -v "^mode" $O/ab.txt
