#!/bin/bash
# MSM sort rewrite check: MSM + Groth16 parity tests, skewed-scalar timings, kernel stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-sort}
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_msm_gpu.py tests/test_groth16_gpu.py tests/test_golden_gpu.py "tests/test_configs_full.py::test_msm_bls12377_2p22_vs_oracle" > gpurun_out/${T}_tests.log 2>&1
rc=$?
grep -E "passed|failed" gpurun_out/${T}_tests.log | tail -3
[ $rc -ne 0 ] && { grep -E "FAILED|Error|error" gpurun_out/${T}_tests.log | head -30; tail -40 gpurun_out/${T}_tests.log; exit $rc; }
for s in uniform zero one wire; do timeout -k 10 120 python tools/msm_only.py --scalars $s --reps 5 || exit 1; done
timeout -k 10 120 python tools/msm_only.py --precompute --reps 5 || exit 1
timeout -k 10 200 python tools/msm_only.py --logn 24 --reps 2 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof -o prof -- python3 bench.py --no-cpu-baseline --no-secondary > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -30 gpurun_out/${T}_bench.err; exit 1; }
head -c 1500 gpurun_out/${T}_bench.json; echo
python3 tools/prof_summary.py $(ls gpurun_out/${T}_prof/*kernel_stats.csv gpurun_out/${T}_prof/*/*kernel_stats.csv 2>/dev/null | head -1) > gpurun_out/${T}_prof_summary.txt; head -30 gpurun_out/${T}_prof_summary.txt
