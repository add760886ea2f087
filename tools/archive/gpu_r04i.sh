#!/bin/bash
# r04i: NTT rounds with one mad chain per product (default now) and the DIF round
# twiddles fetched one round ahead (NTT_TW_PF): parity over every NTT / computeH
# consumer, then same-box A/B: default vs GM_NTT_CHAIN=0 vs alt_pf0.so (-DNTT_TW_PF=0).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-r04i}
timeout -k 10 900 python -u -m pytest tests/test_ntt_gpu.py tests/test_golden_gpu.py tests/test_configs_full.py tests/test_groth16_gpu.py tests/test_icicle_replay_gpu.py tests/test_plonk_replay_gpu.py -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
lib_env() {
  unset GNARK_MI355X_LIB GM_NTT_CHAIN
  case $1 in
    nochain) export GM_NTT_CHAIN=0 ;;
    pf0) export GNARK_MI355X_LIB=$PWD/gnark-icicle_amd/alt_pf0.so ;;
  esac
}
for rep in 1 2 3; do
  for v in default nochain pf0; do
    lib_env $v
    for args in "--logn 24" "--logn 24 --coset" "--curve bls12377 --logn 22" "--logn 20"; do
      echo -n "$v ntt $args: "; timeout -k 10 120 python3 tools/ntt_only.py $args || exit 1
    done
  done
done 2>&1 | tee gpurun_out/${T}_ntt_ab.txt | cut -c1-150
for v in default pf0 default pf0; do
  lib_env $v
  timeout -k 10 400 python3 bench.py --no-cpu-baseline --steps 1 --warmup 1 --g16-logn 24 --g16-plain 24 --msm-extra 0 --ntt-logn 20 > gpurun_out/${T}_g16_$v.json 2> gpurun_out/${T}_g16_$v.err || { tail -20 gpurun_out/${T}_g16_$v.err; exit 1; }
  python3 -c "
import json
for g in json.load(open('gpurun_out/${T}_g16_$v.json'))['secondary']['groth16']: print('$v g16 2^%d' % g['logn'], g['pk'], g['prove_ms_host_inputs'], g['prove_ms_device_inputs'], g['prove_ms_r1cs_resident'])" | tee -a gpurun_out/${T}_g16_ab.txt
done
lib_env default
