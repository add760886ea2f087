#!/bin/bash
# r06ad: MSM GPU tests (incl. the wave-stamp test), then the driver bench + rocprof cross-check (r06e.sh)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_msm_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06ad_tests.log 2>&1 || { tail -30 gpurun_out/r06ad_tests.log; exit 1; }
tail -1 gpurun_out/r06ad_tests.log
bash tools/gpu/r06e.sh r06ad
