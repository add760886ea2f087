#!/bin/bash
# r06k: Z plan early on the auxiliary stream (default) vs after K (alt): Groth16 parity, same-box A/B, exposed time
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_groth16_gpu.py tests/test_r1cs_gpu.py tests/test_pk_io_gpu.py tests/test_configs_full.py tests/test_icicle_replay_gpu.py tests/test_reference_r1cs.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06k_tests.log 2>&1 || { tail -30 gpurun_out/r06k_tests.log; exit 1; }
tail -1 gpurun_out/r06k_tests.log
ALT="GNARK_MI355X_LIB=$R/gnark-icicle_amd/libgnark_mi355x_alt.so"
AB_TIMEOUT=200 bash tools/ab_run.sh gpurun_out/r06k_ab.txt 2 "" "$ALT" -- python3 tools/g16_only.py --logn 24 --reps 3 || exit 1
AB_TIMEOUT=300 bash tools/ab_run.sh gpurun_out/r06k_ab.txt 2 "" "$ALT" -- python3 tools/g16_only.py --logn 24 --reps 3 --precompute || exit 1
AB_TIMEOUT=200 bash tools/ab_run.sh gpurun_out/r06k_ab.txt 2 "" "$ALT" -- python3 tools/g16_only.py --logn 20 --reps 5 || exit 1
bash tools/gpu/r06j.sh || exit 1
