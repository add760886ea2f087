#!/bin/bash
# r03p: NTT load/store phases with the element-wise factor products interleaved: NTT / computeH /
# Groth16 / PLONK / replay parity tests, then 2^24 timings alternated against the
# previous commit (alt2.so: HEAD ntt.o).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-r03p}
timeout -k 10 600 python -u -m pytest tests/test_ntt_gpu.py tests/test_golden_gpu.py tests/test_groth16_gpu.py tests/test_plonk_replay_gpu.py tests/test_icicle_replay_gpu.py tests/test_r1cs_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/${T}_tests.log)"
timeout -k 10 600 python -u -m pytest tests/test_configs_full.py -m gpu -x -q --timeout 300 --timeout-method thread -k "ntt" > gpurun_out/${T}_tests_full.log 2>&1 || { tail -40 gpurun_out/${T}_tests_full.log; exit 1; }
echo "full-size ntt: $(tail -1 gpurun_out/${T}_tests_full.log)"
for rep in 1 2 3; do
  for v in new old; do
    unset GNARK_MI355X_LIB
    [ $v = old ] && export GNARK_MI355X_LIB=$PWD/gnark-icicle_amd/alt2.so
    for args in "--logn 24 --reps 4" "--logn 24 --reps 4 --coset" "--curve bls12377 --logn 22 --reps 4"; do
      echo -n "$v ntt $args: "
      timeout -k 10 200 python tools/ntt_only.py $args || exit 1
    done
  done
done > gpurun_out/${T}_ab.txt 2>&1 || { tail -20 gpurun_out/${T}_ab.txt; exit 1; }
cut -c1-140 gpurun_out/${T}_ab.txt
