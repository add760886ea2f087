#!/bin/bash
# G1 accumulation with the merged Y3 reduction: MSM + Groth16 parity tests, G1 MSM timing, default bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_msm_gpu.py tests/test_groth16_gpu.py > gpurun_out/y3_tests.log 2>&1 || { tail -30 gpurun_out/y3_tests.log; exit 1; }
tail -2 gpurun_out/y3_tests.log
timeout -k 10 100 python tools/msm_only.py --reps 5 2>&1 | tee gpurun_out/y3_msm.txt || exit 1
timeout -k 10 100 python tools/msm_only.py --reps 5 --precompute 2>&1 | tee -a gpurun_out/y3_msm.txt || exit 1
timeout -k 10 300 python bench.py > gpurun_out/y3_bench.json 2> gpurun_out/y3_bench.err || { tail -20 gpurun_out/y3_bench.err; exit 1; }
python - <<'PY'
import json
d=json.loads(open("gpurun_out/y3_bench.json").read().strip().splitlines()[-1])
print(d["value"],d["ms_per_step"],d.get("latency_ms"),d["roofline"]["avg_launch_ms"],json.dumps(d["secondary"]["msm"]))
PY
