#!/bin/bash
# r05af: fresh-process 2^24 plain-key host-input proves: host-input buffers + pinned ring reserved at key
# upload (GM_G16_PREPARE_H=2, default) vs tables only (=1); Groth16 / pk-io / R1CS GPU tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05af; mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_pk_io_gpu.py tests/test_groth16_gpu.py tests/test_r1cs_gpu.py tests/test_reference_r1cs.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  for v in 1 2; do
    echo "== prepare_h=$v" >> $O/ab3.txt
    GM_G16_PREPARE_H=$v timeout -k 10 300 python3 tools/g16_host_trace.py >> $O/ab3.txt 2>> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  done
done
cat $O/ab3.txt
