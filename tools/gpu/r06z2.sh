#!/bin/bash
# r06z2: the auxiliary stream at the greatest priority (ap) vs default priority, more reps; trace of ap
# (experiment not kept: its code is not in the tree; the script documents how profiles/r06y_msm_order_aux_prio_ab.txt was measured)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
L=$PWD/gnark-icicle_amd
AB_TIMEOUT=200 bash tools/ab_run.sh gpurun_out/r06z2_ab.txt 3 "" "GNARK_MI355X_LIB=$L/libgnark_mi355x_ap.so" -- python3 tools/g16_only.py --logn 24 --reps 3 > /dev/null || exit 1
AB_TIMEOUT=300 bash tools/ab_run.sh gpurun_out/r06z2_ab.txt 3 "" "GNARK_MI355X_LIB=$L/libgnark_mi355x_ap.so" -- python3 tools/g16_only.py --logn 24 --reps 3 --precompute > /dev/null || exit 1
AB_TIMEOUT=200 bash tools/ab_run.sh gpurun_out/r06z2_ab.txt 2 "" "GNARK_MI355X_LIB=$L/libgnark_mi355x_ap.so" -- python3 tools/g16_only.py --logn 20 --reps 5 > /dev/null || exit 1
sed -E 's#GNARK_MI355X_LIB=[^ ]*/libgnark_mi355x_([a-z0-9]+)\.so#\1#' gpurun_out/r06z2_ab.txt
env GNARK_MI355X_LIB=$L/libgnark_mi355x_ap.so timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r06z2_kt -o kt -- python3 tools/g16_only.py --logn 24 --reps 1 > gpurun_out/r06z2_kt.out 2>&1 || { tail -5 gpurun_out/r06z2_kt.out; exit 1; }
TR=$(find gpurun_out/r06z2_kt -name "*kernel_trace.csv" | head -1)
python3 tools/g16_exposed.py "$TR" | tee gpurun_out/r06z2_exposed.txt
gzip -f "$TR"
