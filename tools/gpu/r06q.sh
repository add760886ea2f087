#!/bin/bash
# r06q: the 2^20 G1 accumulation in ONE round of 3 (r3) / 4 (r4) waves per SIMD (slices of M / threads entries)
# (experiment not kept: its code is not in the tree; the script documents how profiles/r06q_*.txt was measured)
# instead of slices of 32 entries (two rounds at four waves), with three and four (s4) MSMs in flight
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
L=$PWD/gnark-icicle_amd
for v in r3 r4; do
  GNARK_MI355X_LIB=$L/libgnark_mi355x_$v.so timeout -k 10 300 python -u -m pytest tests/test_msm_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "async or bench or uniform or edge or skew or bucket" > gpurun_out/r06q_tests_$v.log 2>&1 || { tail -30 gpurun_out/r06q_tests_$v.log; exit 1; }
  tail -1 gpurun_out/r06q_tests_$v.log
done
AB_TIMEOUT=150 bash tools/ab_run.sh gpurun_out/r06q_ab.txt 3 "" "GNARK_MI355X_LIB=$L/libgnark_mi355x_r3.so" "GNARK_MI355X_LIB=$L/libgnark_mi355x_r4.so" -- python3 bench.py --steps 30 --warmup 5 --no-secondary --no-cpu-baseline > /dev/null || exit 1
python3 - <<'PY'
import json
for l in open("gpurun_out/r06q_ab.txt"):
    tag, js = l.split(" | ", 1)
    d = json.loads(js); r = d["roofline"]
    print(tag.replace("/root/repo/gnark-icicle_amd/", ""), d["value"], d["ms_per_step"], r["avg_launch_ms"], r["isolated"]["avg_launch_ms"], d["latency_ms"])
PY
GNARK_MI355X_LIB=$L/libgnark_mi355x_r3.so timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r06q_kt -o kt -- python3 bench.py --steps 20 --warmup 5 --no-secondary --no-cpu-baseline > gpurun_out/r06q_kt.json 2> gpurun_out/r06q_kt.err || { tail -20 gpurun_out/r06q_kt.err; exit 1; }
gzip -f $(find gpurun_out/r06q_kt -name "*kernel_trace.csv")
