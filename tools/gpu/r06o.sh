#!/bin/bash
# r06o: async accumulations on one stream of their own at normal (acc1) / low (acc2) priority, the sorts and
# (experiment not kept: its code is not in the tree; the script documents how profiles/r06o_*.txt was measured)
# reductions on the high-priority slot streams, vs the accumulation on the slot stream chained by acc_tail (default)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
L=$PWD/gnark-icicle_amd
for v in 1 2; do
  GNARK_MI355X_LIB=$L/libgnark_mi355x_acc$v.so timeout -k 10 300 python -u -m pytest tests/test_msm_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "async or bench or uniform" > gpurun_out/r06o_tests$v.log 2>&1 || { tail -30 gpurun_out/r06o_tests$v.log; exit 1; }
  tail -1 gpurun_out/r06o_tests$v.log
done
AB_TIMEOUT=150 bash tools/ab_run.sh gpurun_out/r06o_ab.txt 4 "" "GNARK_MI355X_LIB=$L/libgnark_mi355x_acc1.so" "GNARK_MI355X_LIB=$L/libgnark_mi355x_acc2.so" -- python3 bench.py --steps 30 --warmup 5 --no-secondary --no-cpu-baseline > /dev/null || exit 1
python3 - <<'PY'
import json
for l in open("gpurun_out/r06o_ab.txt"):
    tag, js = l.split(" | ", 1)
    d = json.loads(js); r = d["roofline"]
    print(tag.replace("/root/repo/gnark-icicle_amd/", ""), d["value"], d["ms_per_step"], r["avg_launch_ms"], r.get("timing_source"), d["latency_ms"])
PY
GNARK_MI355X_LIB=$L/libgnark_mi355x_acc1.so timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r06o_kt -o kt -- python3 bench.py --steps 20 --warmup 5 --no-secondary --no-cpu-baseline > gpurun_out/r06o_kt.json 2> gpurun_out/r06o_kt.err || { tail -20 gpurun_out/r06o_kt.err; exit 1; }
gzip -f $(find gpurun_out/r06o_kt -name "*kernel_trace.csv")
