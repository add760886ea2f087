#!/bin/bash
# r06v: coarse sort bins of the shared-bucket (precomputed) layout: ~1.5K (bs4096) / ~3K (bs8192) entries vs ~0.75K (default)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
L=$PWD/gnark-icicle_amd
for v in 4096 8192; do
  GNARK_MI355X_LIB=$L/libgnark_mi355x_bs$v.so timeout -k 10 600 python -u -m pytest tests/test_msm_gpu.py tests/test_groth16_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "precomp or groth16" > gpurun_out/r06v_tests$v.log 2>&1 || { tail -30 gpurun_out/r06v_tests$v.log; exit 1; }
  tail -1 gpurun_out/r06v_tests$v.log
done
AB_TIMEOUT=300 bash tools/ab_run.sh gpurun_out/r06v_msm.txt 2 "" "GNARK_MI355X_LIB=$L/libgnark_mi355x_bs4096.so" "GNARK_MI355X_LIB=$L/libgnark_mi355x_bs8192.so" -- python3 tools/msm_only.py --logn 24 --reps 5 --precompute > /dev/null || exit 1
AB_TIMEOUT=300 bash tools/ab_run.sh gpurun_out/r06v_msm.txt 1 "" "GNARK_MI355X_LIB=$L/libgnark_mi355x_bs4096.so" "GNARK_MI355X_LIB=$L/libgnark_mi355x_bs8192.so" -- python3 tools/msm_only.py --logn 20 --reps 10 --precompute > /dev/null || exit 1
AB_TIMEOUT=300 bash tools/ab_run.sh gpurun_out/r06v_ab.txt 2 "" "GNARK_MI355X_LIB=$L/libgnark_mi355x_bs4096.so" "GNARK_MI355X_LIB=$L/libgnark_mi355x_bs8192.so" -- python3 tools/g16_only.py --logn 24 --reps 3 --precompute > /dev/null || exit 1
sed -E 's#GNARK_MI355X_LIB=[^ ]*/libgnark_mi355x_([a-z0-9]+)\.so#\1#' gpurun_out/r06v_msm.txt gpurun_out/r06v_ab.txt | cut -c1-240
