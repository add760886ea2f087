#!/bin/bash
# r06w: plain-layout coarse sort bins of ~0.5K entries (GM_SORT_BIN_PLAIN=1024 build, bp1k) vs ~1K (default)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
ALT="GNARK_MI355X_LIB=$PWD/gnark-icicle_amd/libgnark_mi355x_bp1k.so"
env $ALT timeout -k 10 600 python -u -m pytest tests/test_msm_gpu.py tests/test_groth16_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06w_tests.log 2>&1 || { tail -30 gpurun_out/r06w_tests.log; exit 1; }
tail -1 gpurun_out/r06w_tests.log
AB_TIMEOUT=200 bash tools/ab_run.sh gpurun_out/r06w_msm.txt 2 "" "$ALT" -- python3 tools/msm_only.py --logn 24 --reps 5 > /dev/null || exit 1
AB_TIMEOUT=200 bash tools/ab_run.sh gpurun_out/r06w_msm.txt 2 "" "$ALT" -- python3 tools/msm_only.py --logn 22 --reps 5 --glv 0 > /dev/null || exit 1
AB_TIMEOUT=200 bash tools/ab_run.sh gpurun_out/r06w_ab.txt 2 "" "$ALT" -- python3 tools/g16_only.py --logn 24 --reps 3 > /dev/null || exit 1
AB_TIMEOUT=300 bash tools/ab_run.sh gpurun_out/r06w_ab.txt 1 "" "$ALT" -- python3 tools/g16_only.py --logn 24 --reps 3 --precompute > /dev/null || exit 1
sed -E 's#GNARK_MI355X_LIB=[^ ]*/libgnark_mi355x_([a-z0-9]+)\.so#\1#' gpurun_out/r06w_msm.txt gpurun_out/r06w_ab.txt | cut -c1-240
