#!/bin/bash
# r06ai: 2^20 G1 accumulation slices of 16 (k16) / 24 (k24) entries vs 32 (default) in the pipelined bench, now that
# the accumulations are ordered: shorter slices = more, shorter block rounds, so the next MSM's sort kernels find
# wave slots sooner
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
L=$PWD/gnark-icicle_amd
for v in k16 k24; do
  GNARK_MI355X_LIB=$L/libgnark_mi355x_$v.so timeout -k 10 300 python -u -m pytest tests/test_msm_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06ai_tests_$v.log 2>&1 || { tail -30 gpurun_out/r06ai_tests_$v.log; exit 1; }
  tail -1 gpurun_out/r06ai_tests_$v.log
done
AB_TIMEOUT=150 bash tools/ab_run.sh gpurun_out/r06ai_ab.txt 6 "" "GNARK_MI355X_LIB=$L/libgnark_mi355x_k24.so" -- python3 bench.py --steps 30 --warmup 5 --no-secondary --no-cpu-baseline > /dev/null || exit 1
python3 - <<'PY'
import json
for l in open("gpurun_out/r06ai_ab.txt"):
    tag, js = l.split(" | ", 1)
    d = json.loads(js); r = d["roofline"]
    print(tag.split("/")[-1], d["value"], d["ms_per_step"], r["avg_launch_ms"], r["timing_source"], r["isolated"]["avg_launch_ms"], d["latency_ms"])
PY
