#!/bin/bash
# What the driver runs at round end on one GPU: smoke(), then the default bench (timed).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
start=$SECONDS
timeout -k 10 900 python bench.py > gpurun_out/final_bench.json 2> gpurun_out/final_bench.err || { tail -20 gpurun_out/final_bench.err; exit 1; }
echo "default bench wall: $((SECONDS - start)) s"
head -c 600 gpurun_out/final_bench.json; echo
