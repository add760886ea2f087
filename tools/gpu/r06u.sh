#!/bin/bash
# r06u: ~2K-entry coarse sort bins for plain (non-GLV) plans (GM_SORT_BIN_ENTRIES=4096 build, be4k) vs ~1K (default)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
ALT="GNARK_MI355X_LIB=$PWD/gnark-icicle_amd/libgnark_mi355x_be4k.so"
env $ALT timeout -k 10 600 python -u -m pytest tests/test_msm_gpu.py tests/test_groth16_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06u_tests.log 2>&1 || { tail -30 gpurun_out/r06u_tests.log; exit 1; }
tail -1 gpurun_out/r06u_tests.log
AB_TIMEOUT=200 bash tools/ab_run.sh gpurun_out/r06u_msm.txt 2 "" "$ALT" -- python3 tools/msm_only.py --logn 24 --reps 5 > /dev/null || exit 1
AB_TIMEOUT=300 bash tools/ab_run.sh gpurun_out/r06u_msm.txt 2 "" "$ALT" -- python3 tools/msm_only.py --logn 24 --reps 5 --precompute > /dev/null || exit 1
AB_TIMEOUT=200 bash tools/ab_run.sh gpurun_out/r06u_ab.txt 2 "" "$ALT" -- python3 tools/g16_only.py --logn 24 --reps 3 || exit 1
AB_TIMEOUT=300 bash tools/ab_run.sh gpurun_out/r06u_ab.txt 2 "" "$ALT" -- python3 tools/g16_only.py --logn 24 --reps 3 --precompute || exit 1
sed -E 's#GNARK_MI355X_LIB=[^ ]*/libgnark_mi355x_([a-z0-9]+)\.so#\1#' gpurun_out/r06u_msm.txt | cut -c1-250
