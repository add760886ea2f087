#!/bin/bash
# Full GPU pass: whole -m gpu suite (per-test timeout sized for the 2^24 cases), then the default bench.
#   bash tools/gpu_full.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-full}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --durations=15 --timeout 400 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -25 gpurun_out/${TAG}_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -30 gpurun_out/${TAG}_bench.err; exit 1; }
head -c 3000 gpurun_out/${TAG}_bench.json
