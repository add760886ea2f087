#!/bin/bash
# r06n: G2 pair multiply with quad-permutation DPP operand spreads (PF2_QUAD, alt build) vs the committed form
# (experiment not kept: its code is not in the tree; the script documents how profiles/r06n_*.txt was measured)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
ALT="GNARK_MI355X_LIB=$PWD/gnark-icicle_amd/libgnark_mi355x_alt2.so"
env $ALT timeout -k 10 400 python -u -m pytest tests/test_msm_gpu.py tests/test_golden_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "g2 or G2 or groth16" > gpurun_out/r06n_tests.log 2>&1 || { tail -30 gpurun_out/r06n_tests.log; exit 1; }
tail -1 gpurun_out/r06n_tests.log
AB_TIMEOUT=120 bash tools/ab_run.sh gpurun_out/r06n_ab.txt 3 "" "$ALT" -- python3 tools/msm_only.py --g2 --logn 20 --reps 10 > /dev/null || exit 1
AB_TIMEOUT=120 bash tools/ab_run.sh gpurun_out/r06n_ab.txt 2 "" "$ALT" -- python3 tools/msm_only.py --g2 --logn 22 --reps 5 > /dev/null || exit 1
AB_TIMEOUT=200 bash tools/ab_run.sh gpurun_out/r06n_ab.txt 2 "" "$ALT" -- python3 tools/g16_only.py --logn 24 --reps 3 > /dev/null || exit 1
cat gpurun_out/r06n_ab.txt | sed 's/ | .*\(2^[0-9]*[^|]*ms\/MSM\).*/ | \1/'
