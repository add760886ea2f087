#!/bin/bash
# r06ag: G1 bucket fixup / segment-sum kernels compiled for 3 (w3) / 4 (w4) waves per SIMD (GM_RED_WPE; ~30 / 50-250
# (experiment not kept: its code is not in the tree; the script documents how profiles/r06ag_*.txt was measured)
# VGPRs spilled) vs the register allocator's choice (190-194 VGPRs: two waves, default)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
L=$PWD/gnark-icicle_amd
for v in w3 w4; do
  GNARK_MI355X_LIB=$L/libgnark_mi355x_$v.so timeout -k 10 600 python -u -m pytest tests/test_msm_gpu.py tests/test_groth16_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06ag_tests_$v.log 2>&1 || { tail -30 gpurun_out/r06ag_tests_$v.log; exit 1; }
  tail -1 gpurun_out/r06ag_tests_$v.log
done
AB_TIMEOUT=200 bash tools/ab_run.sh gpurun_out/r06ag_msm.txt 2 "" "GNARK_MI355X_LIB=$L/libgnark_mi355x_w3.so" "GNARK_MI355X_LIB=$L/libgnark_mi355x_w4.so" -- python3 tools/msm_only.py --logn 24 --reps 5 > /dev/null || exit 1
AB_TIMEOUT=300 bash tools/ab_run.sh gpurun_out/r06ag_msm.txt 1 "" "GNARK_MI355X_LIB=$L/libgnark_mi355x_w3.so" "GNARK_MI355X_LIB=$L/libgnark_mi355x_w4.so" -- python3 tools/msm_only.py --logn 24 --reps 5 --precompute > /dev/null || exit 1
AB_TIMEOUT=200 bash tools/ab_run.sh gpurun_out/r06ag_msm.txt 1 "" "GNARK_MI355X_LIB=$L/libgnark_mi355x_w3.so" "GNARK_MI355X_LIB=$L/libgnark_mi355x_w4.so" -- python3 tools/msm_only.py --logn 20 --reps 20 > /dev/null || exit 1
AB_TIMEOUT=200 bash tools/ab_run.sh gpurun_out/r06ag_ab.txt 2 "" "GNARK_MI355X_LIB=$L/libgnark_mi355x_w3.so" "GNARK_MI355X_LIB=$L/libgnark_mi355x_w4.so" -- python3 tools/g16_only.py --logn 24 --reps 3 > /dev/null || exit 1
sed -E 's#GNARK_MI355X_LIB=[^ ]*/libgnark_mi355x_([a-z0-9]+)\.so#\1#' gpurun_out/r06ag_msm.txt gpurun_out/r06ag_ab.txt | sed -E 's/msm_accum_g1=[0-9.]+ //; s/msm_convert_points=[0-9.]+ msm_digits=[0-9.]+ //' | cut -c1-220
