#!/bin/bash
# r03f: full -m gpu suite with the Harvey DIT / block-uniform NTT stages and the
# 4-wave G1 accumulation default, then same-box A/B against the previous
# library (alt.so): NTT 2^24, MSMs, Groth16 2^24 prove; then the default bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-r03f}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
for rep in 1 2; do
  for v in new old; do
    unset GNARK_MI355X_LIB
    [ $v = old ] && export GNARK_MI355X_LIB=$PWD/gnark-icicle_amd/alt.so
    for args in "--logn 24 --reps 4" "--logn 24 --reps 4 --coset"; do
      echo -n "$v ntt $args: "
      timeout -k 10 200 python tools/ntt_only.py $args || exit 1
    done
    for args in "--logn 20 --reps 10" "--logn 20 --reps 5 --precompute" "--curve bls12377 --logn 22 --reps 3"; do
      echo -n "$v msm $args: "
      timeout -k 10 200 python tools/msm_only.py $args || exit 1
    done
  done
done > gpurun_out/${T}_ab.txt 2>&1 || { tail -20 gpurun_out/${T}_ab.txt; exit 1; }
cat gpurun_out/${T}_ab.txt | cut -c1-150
for v in new old new old; do
  unset GNARK_MI355X_LIB
  [ $v = old ] && export GNARK_MI355X_LIB=$PWD/gnark-icicle_amd/alt.so
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 1 --warmup 1 --msm-extra 0 --ntt-logn 20 --g16-logn 24 --g16-plain "" > gpurun_out/${T}_g16_$v.json 2> gpurun_out/${T}_g16_$v.err || { tail -20 gpurun_out/${T}_g16_$v.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/${T}_g16_$v.json')); print('$v', [(g.get('scope'), g.get('prove_ms')) for g in d['secondary']['groth16']])"
done
unset GNARK_MI355X_LIB
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -30 gpurun_out/${T}_bench.err; exit 1; }
head -c 600 gpurun_out/${T}_bench.json; echo
