#!/bin/bash
# r06m: computeH queued at the start of the prove (alt) vs after the wire plan (default)
# (experiment not kept: its code is not in the tree; the script documents how profiles/r06m_*.txt was measured)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
mkdir -p gpurun_out && export TMPDIR=/tmp
ALT="GNARK_MI355X_LIB=$R/gnark-icicle_amd/libgnark_mi355x_alt.so"
env $ALT timeout -k 10 600 python -u -m pytest tests/test_groth16_gpu.py tests/test_r1cs_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06m_tests.log 2>&1 || { tail -30 gpurun_out/r06m_tests.log; exit 1; }
tail -1 gpurun_out/r06m_tests.log
AB_TIMEOUT=200 bash tools/ab_run.sh gpurun_out/r06m_ab.txt 2 "" "$ALT" -- python3 tools/g16_only.py --logn 24 --reps 3 || exit 1
AB_TIMEOUT=300 bash tools/ab_run.sh gpurun_out/r06m_ab.txt 2 "" "$ALT" -- python3 tools/g16_only.py --logn 24 --reps 3 --precompute || exit 1
AB_TIMEOUT=200 bash tools/ab_run.sh gpurun_out/r06m_ab.txt 2 "" "$ALT" -- python3 tools/g16_only.py --logn 20 --reps 5 || exit 1
