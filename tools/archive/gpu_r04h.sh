#!/bin/bash
# r04h: parity of the carry-free product-operand subtractions (NTT rounds, G1 Y3),
# the FP64-limb Montgomery microbench (round toward zero), then same-box A/Bs:
# default vs alt_chain.so (one mad chain per product column, -DGM_FE_CHAIN=1) vs
# alt_difw3.so (DIF radix-4 pass at three waves, -DNTT_DIF_WPE=3).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-r04h}
timeout -k 10 900 python -u -m pytest tests/test_ntt_gpu.py tests/test_golden_gpu.py tests/test_msm_gpu.py tests/test_configs_full.py -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -o /tmp/fp64mont tools/microbench/fp64mont.hip && timeout -k 10 60 /tmp/fp64mont /tmp/fp64mont_dump.txt > gpurun_out/${T}_fp64mont.txt 2>&1 && python3 tools/microbench/fp64mont_check.py /tmp/fp64mont_dump.txt >> gpurun_out/${T}_fp64mont.txt; cat gpurun_out/${T}_fp64mont.txt
lib_env() {
  case $1 in
    chain) export GNARK_MI355X_LIB=$PWD/gnark-icicle_amd/alt_chain.so ;;
    difw3) export GNARK_MI355X_LIB=$PWD/gnark-icicle_amd/alt_difw3.so ;;
    *) unset GNARK_MI355X_LIB ;;
  esac
}
for rep in 1 2 3; do
  for lib in default chain difw3; do
    lib_env $lib
    for args in "--logn 24" "--logn 24 --coset" "--curve bls12377 --logn 22"; do
      echo -n "$lib ntt $args: "; timeout -k 10 120 python3 tools/ntt_only.py $args || exit 1
    done
  done
done 2>&1 | tee gpurun_out/${T}_ntt_ab.txt | cut -c1-150
for rep in 1 2; do
  for lib in default chain; do
    lib_env $lib
    for args in "--logn 20" "--logn 24 --precompute" "--g2 --logn 20" "--curve bls12377 --logn 22" "--curve bls12377 --g2 --logn 22"; do
      echo -n "$lib $args: "; timeout -k 10 200 python3 tools/msm_only.py $args --reps 5 || exit 1
    done
  done
done 2>&1 | tee gpurun_out/${T}_msm_ab.txt | cut -c1-150
for lib in default chain difw3 default chain difw3; do
  lib_env $lib
  timeout -k 10 400 python3 bench.py --no-cpu-baseline --steps 1 --warmup 1 --g16-logn 24 --g16-plain 24 --g16-no-precomputed --msm-extra 0 --ntt-logn 20 > gpurun_out/${T}_g16_$lib.json 2> gpurun_out/${T}_g16_$lib.err || { tail -20 gpurun_out/${T}_g16_$lib.err; exit 1; }
  python3 -c "
import json; g=[x for x in json.load(open('gpurun_out/${T}_g16_$lib.json'))['secondary']['groth16'] if x['logn']==24][0]; print('$lib g16 2^24', g['pk'], g['prove_ms_host_inputs'], g['prove_ms_device_inputs'])" | tee -a gpurun_out/${T}_g16_ab.txt
done
unset GNARK_MI355X_LIB
