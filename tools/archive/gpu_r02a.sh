#!/bin/bash
# Round-2 GPU pass A: full GPU suite (incl. the full-size config tests, progress
# on stdout via -s), then MSM A/Bs and SQ counter passes for the accumulation.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r02a}
timeout -k 10 1100 python -u -m pytest tests -m gpu -v -s --timeout 700 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/${T}_tests.log | tail -25
echo "pytest rc=$rc"
exit $rc
