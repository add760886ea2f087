#!/bin/bash
# r06a: accumulation chain A/B (GM_MSM_ACC_SERIAL) + async MSM tests + rocprof of the bench loop
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
GM_MSM_ACC_SERIAL=1 timeout -k 10 300 python -u -m pytest tests/test_msm_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "async or bench or uniform" > gpurun_out/r06a_tests.log 2>&1 || { tail -30 gpurun_out/r06a_tests.log; exit 1; }
tail -3 gpurun_out/r06a_tests.log
AB_TIMEOUT=150 bash tools/ab_run.sh gpurun_out/r06a_ab.txt 3 "" "GM_MSM_ACC_SERIAL=1" -- python3 bench.py --steps 20 --warmup 5 --no-secondary --no-cpu-baseline > /dev/null || exit 1
python3 - <<'PY'
import json
for l in open("gpurun_out/r06a_ab.txt"):
    tag, js = l.split(" | ", 1)
    d = json.loads(js); r = d["roofline"]
    print(tag, d["value"], d["ms_per_step"], r["avg_launch_ms"], r.get("timing_source"), r["isolated"]["avg_launch_ms"])
PY
GM_MSM_ACC_SERIAL=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06a_prof -o prof -- python3 bench.py --steps 20 --warmup 5 --no-secondary --no-cpu-baseline > gpurun_out/r06a_profbench.json 2> gpurun_out/r06a_prof.err || { tail -30 gpurun_out/r06a_prof.err; exit 1; }
T=$(find gpurun_out/r06a_prof -name "*kernel_trace.csv" | head -1)
python3 tools/prof_trace_summary.py "$T" --last 20 > gpurun_out/r06a_trace_summary.txt
head -12 gpurun_out/r06a_trace_summary.txt
python3 -c "import json; d=json.load(open('gpurun_out/r06a_profbench.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], r['avg_launch_ms'], r['timing_source'])"
rm -f "$T"
