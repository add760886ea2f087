#!/bin/bash
# r03x: the driver's default N=1 bench invocation on the final tree.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-r03x}
start=$(date +%s)
timeout -k 10 900 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -30 gpurun_out/${T}_bench.err; exit 1; }
echo "elapsed $(( $(date +%s) - start )) s"
head -c 500 gpurun_out/${T}_bench.json; echo
