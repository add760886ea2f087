#!/bin/bash
# One GPU-box pass: parity tests, bench line, rocprof kernel summary, PMC traffic.
#   bash tools/gpu_check.sh TAG [tests|notests]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-run}
if [ "${2:-tests}" = tests ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
  tail -3 gpurun_out/${TAG}_tests.log
fi
timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -30 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
# primary bench kernels only (their averages must agree with the bench line's HIP-event figures)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o prof -- python3 bench.py --no-cpu-baseline --no-secondary > gpurun_out/${TAG}_profbench.json 2> gpurun_out/${TAG}_prof.err || { tail -30 gpurun_out/${TAG}_prof.err; exit 1; }
# Groth16 2^24 (precomputed) kernel timeline
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_g16 -o prof -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 1 --g16-logn 24 --g16-plain "" --msm-extra 0 --ntt-logn 20 > gpurun_out/${TAG}_g16.json 2> gpurun_out/${TAG}_g16.err || { tail -30 gpurun_out/${TAG}_g16.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_pmcf -o pmc -- python3 bench.py --no-cpu-baseline --no-secondary --steps 2 --warmup 1 > /dev/null 2> gpurun_out/${TAG}_pmcf.err || { tail -20 gpurun_out/${TAG}_pmcf.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${TAG}_pmcw -o pmc -- python3 bench.py --no-cpu-baseline --no-secondary --steps 2 --warmup 1 > /dev/null 2> gpurun_out/${TAG}_pmcw.err || { tail -20 gpurun_out/${TAG}_pmcw.err; exit 1; }
python3 tools/pmc_traffic.py gpurun_out/${TAG}_pmcf gpurun_out/${TAG}_pmcw gpurun_out/${TAG}_pmc_traffic.json > /dev/null
echo done
