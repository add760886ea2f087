#!/bin/bash
# Round-3 baseline: full -m gpu suite, smoke, default bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r03base}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --durations=25 --timeout 400 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -3 gpurun_out/${T}_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -30 gpurun_out/${T}_bench.err; exit 1; }
head -c 600 gpurun_out/${T}_bench.json; echo
