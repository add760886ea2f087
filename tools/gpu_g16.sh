#!/bin/bash
# Groth16 parity tests + a rocprofv3 kernel timeline of the 2^24 precomputed prove.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=${1:-g16}
if [ "${2:-}" != notests ]; then timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "groth16" > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }; fi
[ "${2:-}" != notests ] && tail -2 gpurun_out/${TAG}_tests.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o prof -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 1 --g16-logn 24 --g16-plain "" --msm-extra 0 --ntt-logn 20 > gpurun_out/${TAG}.json 2> gpurun_out/${TAG}.err || { tail -30 gpurun_out/${TAG}.err; exit 1; }
python3 -c "import json; print(json.load(open('gpurun_out/${TAG}.json'))['secondary']['groth16'])"
python3 tools/g16_timeline.py $(ls gpurun_out/${TAG}_prof/prof_kernel_trace.csv gpurun_out/${TAG}_prof/*/*kernel_trace.csv 2>/dev/null | head -1) > gpurun_out/${TAG}_timeline.txt; head -40 gpurun_out/${TAG}_timeline.txt
