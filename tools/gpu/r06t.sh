#!/bin/bash
# r06t: no bucket memset (empty buckets read as infinity in the segment sums) + capped split-bin sort grids, vs the
# previous library (base); GPU tests of the MSM / Groth16 paths with the new library first
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
BASE="GNARK_MI355X_LIB=$PWD/gnark-icicle_amd/libgnark_mi355x_base.so"
timeout -k 10 900 python -u -m pytest tests/test_msm_gpu.py tests/test_groth16_gpu.py tests/test_r1cs_gpu.py tests/test_golden_gpu.py tests/test_icicle_replay_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06t_tests.log 2>&1 || { tail -30 gpurun_out/r06t_tests.log; exit 1; }
tail -1 gpurun_out/r06t_tests.log
AB_TIMEOUT=150 bash tools/ab_run.sh gpurun_out/r06t_bench_ab.txt 3 "" "$BASE" -- python3 bench.py --steps 30 --warmup 5 --no-secondary --no-cpu-baseline > /dev/null || exit 1
AB_TIMEOUT=200 bash tools/ab_run.sh gpurun_out/r06t_ab.txt 2 "" "$BASE" -- python3 tools/g16_only.py --logn 24 --reps 3 || exit 1
AB_TIMEOUT=300 bash tools/ab_run.sh gpurun_out/r06t_ab.txt 2 "" "$BASE" -- python3 tools/g16_only.py --logn 24 --reps 3 --precompute || exit 1
AB_TIMEOUT=200 bash tools/ab_run.sh gpurun_out/r06t_ab.txt 2 "" "$BASE" -- python3 tools/g16_only.py --logn 20 --reps 5 || exit 1
python3 - <<'PY'
import json
for l in open("gpurun_out/r06t_bench_ab.txt"):
    tag, js = l.split(" | ", 1)
    d = json.loads(js); r = d["roofline"]
    print(tag.split("/")[-1], d["value"], d["ms_per_step"], r["avg_launch_ms"], r["isolated"]["avg_launch_ms"], d["latency_ms"])
PY
