#!/bin/bash
# r06z: the auxiliary stream (computeH) at the greatest stream priority (GM_AUX_PRIO=1 build, ap), and with the
# (experiment not kept: its code is not in the tree; the script documents how profiles/r06y_msm_order_aux_prio_ab.txt was measured)
# r06y order + early Z plan (apo2), vs default priority (default)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
L=$PWD/gnark-icicle_amd
env GNARK_MI355X_LIB=$L/libgnark_mi355x_apo2.so timeout -k 10 600 python -u -m pytest tests/test_groth16_gpu.py tests/test_r1cs_gpu.py tests/test_ntt_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06z_tests.log 2>&1 || { tail -30 gpurun_out/r06z_tests.log; exit 1; }
tail -1 gpurun_out/r06z_tests.log
AB_TIMEOUT=200 bash tools/ab_run.sh gpurun_out/r06z_ab.txt 2 "" "GNARK_MI355X_LIB=$L/libgnark_mi355x_ap.so" "GNARK_MI355X_LIB=$L/libgnark_mi355x_apo2.so" -- python3 tools/g16_only.py --logn 24 --reps 3 > /dev/null || exit 1
AB_TIMEOUT=300 bash tools/ab_run.sh gpurun_out/r06z_ab.txt 2 "" "GNARK_MI355X_LIB=$L/libgnark_mi355x_ap.so" "GNARK_MI355X_LIB=$L/libgnark_mi355x_apo2.so" -- python3 tools/g16_only.py --logn 24 --reps 3 --precompute > /dev/null || exit 1
sed -E 's#GNARK_MI355X_LIB=[^ ]*/libgnark_mi355x_([a-z0-9]+)\.so#\1#' gpurun_out/r06z_ab.txt
env GNARK_MI355X_LIB=$L/libgnark_mi355x_apo2.so timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r06z_kt -o kt -- python3 tools/g16_only.py --logn 24 --reps 1 > gpurun_out/r06z_kt.out 2>&1 || { tail -5 gpurun_out/r06z_kt.out; exit 1; }
TR=$(find gpurun_out/r06z_kt -name "*kernel_trace.csv" | head -1)
python3 tools/g16_exposed.py "$TR" | tee gpurun_out/r06z_exposed.txt
gzip -f "$TR"
