#!/bin/bash
# r06ae: bench with the accumulation's wave stamps (default; second run: 64 stamp pairs per launch; third: entry stamps from the first 64 blocks only) vs without them (GM_WAVE_STAMPS=0 build, ns): do the
# stamps' per-wave atomics cost the profiled timed loop anything?
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_msm_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "stamps or async or bench" > gpurun_out/r06ae_tests.log 2>&1 || { tail -30 gpurun_out/r06ae_tests.log; exit 1; }
tail -1 gpurun_out/r06ae_tests.log
AB_TIMEOUT=150 bash tools/ab_run.sh gpurun_out/r06ae_ab.txt 4 "" "GNARK_MI355X_LIB=$PWD/gnark-icicle_amd/libgnark_mi355x_ns.so" -- python3 bench.py --steps 30 --warmup 5 --no-secondary --no-cpu-baseline > /dev/null || exit 1
python3 - <<'PY'
import json
for l in open("gpurun_out/r06ae_ab.txt"):
    tag, js = l.split(" | ", 1)
    d = json.loads(js); r = d["roofline"]
    print(tag.split("/")[-1], d["value"], d["ms_per_step"], r["avg_launch_ms"], r["timing_source"], r["isolated"]["avg_launch_ms"], d["latency_ms"])
PY
