#!/bin/bash
# r06l: async MSM point conversion on a helper stream of its slot (GM_MSM_CONV_STREAM=1) vs on the slot stream
# (experiment not kept: its code is not in the tree; the script documents how profiles/r06l_*.txt was measured)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
GM_MSM_CONV_STREAM=1 timeout -k 10 300 python -u -m pytest tests/test_msm_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "async or bench or uniform" > gpurun_out/r06l_tests.log 2>&1 || { tail -30 gpurun_out/r06l_tests.log; exit 1; }
tail -1 gpurun_out/r06l_tests.log
AB_TIMEOUT=150 bash tools/ab_run.sh gpurun_out/r06l_ab.txt 4 "" "GM_MSM_CONV_STREAM=1" -- python3 bench.py --steps 30 --warmup 5 --no-secondary --no-cpu-baseline > /dev/null || exit 1
python3 - <<'PY'
import json
for l in open("gpurun_out/r06l_ab.txt"):
    tag, js = l.split(" | ", 1)
    d = json.loads(js); r = d["roofline"]
    print(tag, d["value"], d["ms_per_step"], r["avg_launch_ms"], r.get("timing_source"), d["latency_ms"])
PY
GM_MSM_CONV_STREAM=1 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r06l_kt -o kt -- python3 bench.py --steps 20 --warmup 5 --no-secondary --no-cpu-baseline > gpurun_out/r06l_kt.json 2> gpurun_out/r06l_kt.err || { tail -20 gpurun_out/r06l_kt.err; exit 1; }
gzip -f $(find gpurun_out/r06l_kt -name "*kernel_trace.csv")
