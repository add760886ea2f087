#!/bin/bash
# r03y: BN254 G2 pair add with Y3 = R W - Y1 PPP as one four-product reduction:
# MSM / Groth16 parity, then alternated timings vs the previous commit (alt3.so).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-r03y}
timeout -k 10 600 python -u -m pytest tests/test_msm_gpu.py tests/test_groth16_gpu.py tests/test_configs_full.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/${T}_tests.log)"
for rep in 1 2 3; do
  for v in new old; do
    unset GNARK_MI355X_LIB
    [ $v = old ] && export GNARK_MI355X_LIB=$PWD/gnark-icicle_amd/alt3.so
    for args in "--g2 --logn 20 --reps 5" "--g2 --logn 20 --reps 5 --precompute"; do
      echo -n "$v $args: "
      timeout -k 10 200 python tools/msm_only.py $args || exit 1
    done
  done
done > gpurun_out/${T}_ab.txt 2>&1 || { tail -20 gpurun_out/${T}_ab.txt; exit 1; }
unset GNARK_MI355X_LIB
cut -c1-150 gpurun_out/${T}_ab.txt
for v in new old new old; do
  unset GNARK_MI355X_LIB
  [ $v = old ] && export GNARK_MI355X_LIB=$PWD/gnark-icicle_amd/alt3.so
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 1 --warmup 1 --msm-extra 0 --ntt-logn 20 --g16-logn 24 --g16-plain "" > gpurun_out/${T}_g16_$v.json 2> gpurun_out/${T}_g16_$v.err || { tail -20 gpurun_out/${T}_g16_$v.err; exit 1; }
  python3 -c "
import json; g=json.load(open('gpurun_out/${T}_g16_$v.json'))['secondary']['groth16'][0]; print('g16 $v', g['prove_ms_host_inputs'], g['prove_ms_device_inputs'], g['prove_ms_r1cs_resident'])"
done
