#!/bin/bash
# r06ak: G1 accumulation slices of 32 (kl32) / 48 (kl48) entries for the MSMs above 2^25 entries (the 2^24 Groth16
# (experiment not kept: its code is not in the tree; the script documents how profiles/r06ak_*.txt was measured)
# G1 MSMs) vs 64 (default)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
L=$PWD/gnark-icicle_amd
GNARK_MI355X_LIB=$L/libgnark_mi355x_kl32.so timeout -k 10 600 python -u -m pytest tests/test_msm_gpu.py tests/test_groth16_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06ak_tests.log 2>&1 || { tail -30 gpurun_out/r06ak_tests.log; exit 1; }
tail -1 gpurun_out/r06ak_tests.log
AB_TIMEOUT=200 bash tools/ab_run.sh gpurun_out/r06ak_ab.txt 2 "" "GNARK_MI355X_LIB=$L/libgnark_mi355x_kl32.so" "GNARK_MI355X_LIB=$L/libgnark_mi355x_kl48.so" -- python3 tools/g16_only.py --logn 24 --reps 3 > /dev/null || exit 1
AB_TIMEOUT=300 bash tools/ab_run.sh gpurun_out/r06ak_ab.txt 2 "" "GNARK_MI355X_LIB=$L/libgnark_mi355x_kl32.so" "GNARK_MI355X_LIB=$L/libgnark_mi355x_kl48.so" -- python3 tools/g16_only.py --logn 24 --reps 3 --precompute > /dev/null || exit 1
sed -E 's#GNARK_MI355X_LIB=[^ ]*/libgnark_mi355x_([a-z0-9]+)\.so#\1#' gpurun_out/r06ak_ab.txt | cut -c1-200
