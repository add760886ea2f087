#!/bin/bash
# r06aa: final sort pass in 256-thread blocks with a 3,072-entry stage where bins hold ~1-2K entries (new = default)
# (experiment not kept: its code is not in the tree; the script documents how profiles/r06aa_*.txt was measured)
# vs 1024-thread blocks with a 6,144-entry stage everywhere (base = previous library)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
BASE="GNARK_MI355X_LIB=$PWD/gnark-icicle_amd/libgnark_mi355x_base.so"
timeout -k 10 900 python -u -m pytest tests/test_msm_gpu.py tests/test_groth16_gpu.py tests/test_r1cs_gpu.py tests/test_golden_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06aa_tests.log 2>&1 || { tail -30 gpurun_out/r06aa_tests.log; exit 1; }
tail -1 gpurun_out/r06aa_tests.log
AB_TIMEOUT=200 bash tools/ab_run.sh gpurun_out/r06aa_msm.txt 2 "" "$BASE" -- python3 tools/msm_only.py --logn 24 --reps 5 > /dev/null || exit 1
AB_TIMEOUT=300 bash tools/ab_run.sh gpurun_out/r06aa_msm.txt 2 "" "$BASE" -- python3 tools/msm_only.py --logn 24 --reps 5 --precompute > /dev/null || exit 1
AB_TIMEOUT=200 bash tools/ab_run.sh gpurun_out/r06aa_msm.txt 2 "" "$BASE" -- python3 tools/msm_only.py --logn 22 --reps 5 --glv 0 > /dev/null || exit 1
AB_TIMEOUT=200 bash tools/ab_run.sh gpurun_out/r06aa_ab.txt 2 "" "$BASE" -- python3 tools/g16_only.py --logn 24 --reps 3 > /dev/null || exit 1
AB_TIMEOUT=300 bash tools/ab_run.sh gpurun_out/r06aa_ab.txt 2 "" "$BASE" -- python3 tools/g16_only.py --logn 24 --reps 3 --precompute > /dev/null || exit 1
sed -E 's#GNARK_MI355X_LIB=[^ ]*/libgnark_mi355x_([a-z0-9]+)\.so#\1#' gpurun_out/r06aa_msm.txt gpurun_out/r06aa_ab.txt | sed -E 's/msm_accum_g1=[0-9.]+ msm_bucket_reduce=[0-9.]+ //' | cut -c1-200
