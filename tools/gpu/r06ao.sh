#!/bin/bash
# r06ao: BN254 G2 accumulation slices of 32 (g2k32) / 48 (g2k48) entries for G2 MSMs <= 2^25 entries vs 64 (default)
# (experiment not kept: its code is not in the tree; the script documents how profiles/r06ao_*.txt was measured)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
L=$PWD/gnark-icicle_amd
GNARK_MI355X_LIB=$L/libgnark_mi355x_g2k32.so timeout -k 10 600 python -u -m pytest tests/test_msm_gpu.py tests/test_groth16_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06ao_tests.log 2>&1 || { tail -30 gpurun_out/r06ao_tests.log; exit 1; }
tail -1 gpurun_out/r06ao_tests.log
AB_TIMEOUT=200 bash tools/ab_run.sh gpurun_out/r06ao_ab.txt 3 "" "GNARK_MI355X_LIB=$L/libgnark_mi355x_g2k32.so" "GNARK_MI355X_LIB=$L/libgnark_mi355x_g2k48.so" -- python3 tools/msm_only.py --g2 --logn 20 --reps 10 > /dev/null || exit 1
AB_TIMEOUT=200 bash tools/ab_run.sh gpurun_out/r06ao_ab.txt 2 "" "GNARK_MI355X_LIB=$L/libgnark_mi355x_g2k32.so" "GNARK_MI355X_LIB=$L/libgnark_mi355x_g2k48.so" -- python3 tools/g16_only.py --logn 20 --reps 7 > /dev/null || exit 1
sed -E 's#GNARK_MI355X_LIB=[^ ]*/libgnark_mi355x_([a-z0-9]+)\.so#\1#' gpurun_out/r06ao_ab.txt | sed -E 's/\| msm_accum_g2=([0-9.]+).*/| accum \1/' | cut -c1-200
