#!/bin/bash
# r04ac: sanity after the gm_destroy reorder -- smoke, MSM + Groth16 GPU tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 900 python -u -m pytest tests/test_msm_gpu.py tests/test_groth16_gpu.py tests/test_plonk_replay_gpu.py -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r04ac_tests.log 2>&1 || { tail -40 gpurun_out/r04ac_tests.log; exit 1; }
tail -1 gpurun_out/r04ac_tests.log
