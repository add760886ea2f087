#!/bin/bash
# r06d: NTT butterfly strict chains (alt) and big-MSM slice K=128 (alt2) -- same-box A/Bs + parity
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
mkdir -p gpurun_out && export TMPDIR=/tmp
ALT="GNARK_MI355X_LIB=$R/gnark-icicle_amd/libgnark_mi355x_alt.so"
ALT2="GNARK_MI355X_LIB=$R/gnark-icicle_amd/libgnark_mi355x_alt2.so"
AB_TIMEOUT=120 bash tools/ab_run.sh gpurun_out/r06d_ntt_ab.txt 3 "" "$ALT" -- python3 tools/ntt_only.py --logn 24 --reps 10 || exit 1
AB_TIMEOUT=120 bash tools/ab_run.sh gpurun_out/r06d_ntt_ab.txt 2 "" "$ALT" -- python3 tools/ntt_only.py --logn 24 --reps 10 --coset || exit 1
AB_TIMEOUT=200 bash tools/ab_run.sh gpurun_out/r06d_g16_ab.txt 2 "" "$ALT2" -- python3 tools/g16_only.py --logn 24 --reps 3 || exit 1
AB_TIMEOUT=300 bash tools/ab_run.sh gpurun_out/r06d_g16_ab.txt 2 "" "$ALT2" -- python3 tools/g16_only.py --logn 24 --reps 3 --precompute || exit 1
env $ALT timeout -k 10 300 python -u -m pytest tests/test_ntt_gpu.py tests/test_configs_full.py -m gpu -x -q --timeout 200 --timeout-method thread -k "ntt or compute_h" > gpurun_out/r06d_alt_tests.log 2>&1 || { tail -20 gpurun_out/r06d_alt_tests.log; exit 1; }
tail -2 gpurun_out/r06d_alt_tests.log
env $ALT2 timeout -k 10 400 python -u -m pytest tests/test_configs_full.py -m gpu -x -q --timeout 300 --timeout-method thread -k "2p24" > gpurun_out/r06d_alt2_tests.log 2>&1 || { tail -20 gpurun_out/r06d_alt2_tests.log; exit 1; }
tail -2 gpurun_out/r06d_alt2_tests.log
