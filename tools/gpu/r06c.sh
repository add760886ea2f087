#!/bin/bash
# r06c: pruned library -- whole -m gpu suite, smoke, accumulation-chain A/B, staged-overhead diagnostic
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --durations=15 --timeout 400 --timeout-method thread > gpurun_out/r06c_tests.log 2>&1 || { tail -40 gpurun_out/r06c_tests.log; exit 1; }
tail -4 gpurun_out/r06c_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
AB_TIMEOUT=150 bash tools/ab_run.sh gpurun_out/r06c_ab.txt 3 "" "GM_MSM_ACC_SERIAL=1" -- python3 bench.py --steps 20 --warmup 5 --no-secondary --no-cpu-baseline > /dev/null || exit 1
python3 - <<'PY'
import json
for l in open("gpurun_out/r06c_ab.txt"):
    tag, js = l.split(" | ", 1)
    d = json.loads(js); r = d["roofline"]
    print(tag, d["value"], d["ms_per_step"], r["avg_launch_ms"], r.get("timing_source"), r["isolated"]["avg_launch_ms"])
PY
timeout -k 10 300 python3 tools/staged_overhead.py 20 5 50 | tee gpurun_out/r06c_staged_overhead.txt
