#!/bin/bash
# r06aj: K = 24 (default now) vs 32 (k32) for the other G1 MSMs of <= 2^25 entries: Groth16 2^20 (plain, precomputed),
# precomputed 2^20 MSM, plain 2^22 MSM
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
K32="GNARK_MI355X_LIB=$PWD/gnark-icicle_amd/libgnark_mi355x_k32.so"
timeout -k 10 600 python -u -m pytest tests/test_msm_gpu.py tests/test_groth16_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06aj_tests.log 2>&1 || { tail -30 gpurun_out/r06aj_tests.log; exit 1; }
tail -1 gpurun_out/r06aj_tests.log
AB_TIMEOUT=200 bash tools/ab_run.sh gpurun_out/r06aj_ab.txt 3 "" "$K32" -- python3 tools/g16_only.py --logn 20 --reps 7 > /dev/null || exit 1
AB_TIMEOUT=200 bash tools/ab_run.sh gpurun_out/r06aj_ab.txt 3 "" "$K32" -- python3 tools/g16_only.py --logn 20 --reps 7 --precompute > /dev/null || exit 1
AB_TIMEOUT=200 bash tools/ab_run.sh gpurun_out/r06aj_ab.txt 2 "" "$K32" -- python3 tools/msm_only.py --logn 20 --reps 20 --precompute > /dev/null || exit 1
AB_TIMEOUT=200 bash tools/ab_run.sh gpurun_out/r06aj_ab.txt 2 "" "$K32" -- python3 tools/msm_only.py --logn 20 --reps 20 > /dev/null || exit 1
sed -E 's#GNARK_MI355X_LIB=[^ ]*/libgnark_mi355x_([a-z0-9]+)\.so#\1#' gpurun_out/r06aj_ab.txt | cut -c1-200
