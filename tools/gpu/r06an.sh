#!/bin/bash
# r06an: 2^20 G1 accumulation slices of 20 (k20) / 28 (k28) entries vs 24 (default) in the pipelined bench
# (the k20 / k28 builds were alternative libraries; 24 is the tree's value)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
L=$PWD/gnark-icicle_amd
for v in k20 k28; do
  GNARK_MI355X_LIB=$L/libgnark_mi355x_$v.so timeout -k 10 300 python -u -m pytest tests/test_msm_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06an_tests_$v.log 2>&1 || { tail -30 gpurun_out/r06an_tests_$v.log; exit 1; }
  tail -1 gpurun_out/r06an_tests_$v.log
done
AB_TIMEOUT=150 bash tools/ab_run.sh gpurun_out/r06an_ab.txt 5 "" "GNARK_MI355X_LIB=$L/libgnark_mi355x_k20.so" "GNARK_MI355X_LIB=$L/libgnark_mi355x_k28.so" -- python3 bench.py --steps 30 --warmup 5 --no-secondary --no-cpu-baseline > /dev/null || exit 1
python3 - <<'PY'
import json
for l in open("gpurun_out/r06an_ab.txt"):
    tag, js = l.split(" | ", 1)
    d = json.loads(js); r = d["roofline"]
    print(tag.split("/")[-1], d["value"], d["ms_per_step"], r["avg_launch_ms"], r["timing_source"], r["isolated"]["avg_launch_ms"], d["latency_ms"])
PY
