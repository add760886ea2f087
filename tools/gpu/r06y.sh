#!/bin/bash
# r06y: MSM order A, B, K, B2, Z with Z's digits / sort queued on the auxiliary stream after computeH (third slot,
# (experiment not kept: its code is not in the tree; the script documents how profiles/r06y_msm_order_aux_prio_ab.txt was measured)
# GM_G16_ORDER2=1 build, device-input proves) vs A, B, B2, K, Z with Z planned on the prove's stream (default)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
ALT="GNARK_MI355X_LIB=$PWD/gnark-icicle_amd/libgnark_mi355x_o2.so"
env $ALT timeout -k 10 600 python -u -m pytest tests/test_groth16_gpu.py tests/test_r1cs_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06y_tests.log 2>&1 || { tail -30 gpurun_out/r06y_tests.log; exit 1; }
tail -1 gpurun_out/r06y_tests.log
AB_TIMEOUT=200 bash tools/ab_run.sh gpurun_out/r06y_ab.txt 2 "" "$ALT" -- python3 tools/g16_only.py --logn 24 --reps 3 || exit 1
AB_TIMEOUT=300 bash tools/ab_run.sh gpurun_out/r06y_ab.txt 2 "" "$ALT" -- python3 tools/g16_only.py --logn 24 --reps 3 --precompute || exit 1
AB_TIMEOUT=200 bash tools/ab_run.sh gpurun_out/r06y_ab.txt 2 "" "$ALT" -- python3 tools/g16_only.py --logn 20 --reps 5 || exit 1
env $ALT timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r06y_kt -o kt -- python3 tools/g16_only.py --logn 24 --reps 1 > gpurun_out/r06y_kt.out 2>&1 || { tail -5 gpurun_out/r06y_kt.out; exit 1; }
TR=$(find gpurun_out/r06y_kt -name "*kernel_trace.csv" | head -1)
python3 tools/g16_exposed.py "$TR" | tee gpurun_out/r06y_exposed.txt
gzip -f "$TR"
