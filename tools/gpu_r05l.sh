#!/bin/bash
# r05l: Groth16 GPU tests with the incremental host-input computeH, then a same-box A/B of
# 2^24 host-input proves: old (all three vectors before computeH, one fill thread) vs new.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05l; mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_groth16_gpu.py tests/test_r1cs_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for rep in 1 2; do
  for v in old thr1 inc1 new; do
    case $v in
      old) E="GM_G16_H_INCREMENTAL=0 GM_G16_H2D_THREADS=1";;
      thr1) E="GM_G16_H2D_THREADS=1";;
      inc1) E="GM_G16_H_INCREMENTAL=0";;
      new) E="";;
    esac
    echo "== $v ($E) rep $rep" >> $O/ab.txt
    env $E timeout -k 10 300 python3 tools/g16_host_trace.py device >> $O/ab.txt 2>> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  done
done
cat $O/ab.txt
