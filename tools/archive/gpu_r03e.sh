#!/bin/bash
# r03e: full -m gpu suite on the G1 / G2-pair add trims (carry-free digit sign on S2, one
# borrow chain for X3), then same-box A/B vs the previous library (alt.so) and
# the four-waves-per-SIMD accumulation variants, then the default bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-r03e}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
for rep in 1 2; do
  for v in new old w4 w4np; do
    unset GNARK_MI355X_LIB GM_MSM_ACCUM
    [ $v = old ] && export GNARK_MI355X_LIB=$PWD/gnark-icicle_amd/alt.so
    [ $v = w4 ] && export GM_MSM_ACCUM=w4
    [ $v = w4np ] && export GM_MSM_ACCUM=w4np
    ARGS=("--logn 20 --reps 10" "--logn 20 --reps 5 --precompute")
    case $v in new|old) ARGS+=("--g2 --logn 20 --reps 5" "--curve bls12377 --g2 --logn 22 --reps 2");; esac
    for args in "${ARGS[@]}"; do
      echo -n "$v $args: "
      timeout -k 10 200 python tools/msm_only.py $args || exit 1
    done
  done
done > gpurun_out/${T}_ab.txt 2>&1 || { tail -20 gpurun_out/${T}_ab.txt; exit 1; }
unset GNARK_MI355X_LIB GM_MSM_ACCUM
cat gpurun_out/${T}_ab.txt
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -30 gpurun_out/${T}_bench.err; exit 1; }
head -c 700 gpurun_out/${T}_bench.json; echo
