#!/bin/bash
# Focused GPU pass: MSM/Groth16 parity tests, then the bench line.
#   bash tools/gpu_t2.sh TAG [pytest -k expr]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=${1:-t2}
K=${2:-"precomput or groth16 or msm"}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$K" > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -3 gpurun_out/${TAG}_tests.log
timeout -k 10 500 python -u bench.py --no-cpu-baseline --msm-extra 1 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -30 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
