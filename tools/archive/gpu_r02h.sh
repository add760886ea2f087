#!/bin/bash
# Full GPU suite, then the Groth16 2^24 timeline (tools/gpu_g16.sh, no tests).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r02h_tests.log 2>&1 || { tail -40 gpurun_out/r02h_tests.log; exit 1; }
tail -2 gpurun_out/r02h_tests.log
bash tools/gpu_g16.sh r02h notests
