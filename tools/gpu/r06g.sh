#!/bin/bash
# r06g: edge-parallel fixup (default) vs the per-bucket fixup (alt3): whole -m gpu suite, then same-box A/Bs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --durations=8 --timeout 400 --timeout-method thread > gpurun_out/r06g_tests.log 2>&1 || { tail -40 gpurun_out/r06g_tests.log; exit 1; }
tail -3 gpurun_out/r06g_tests.log
ALT="GNARK_MI355X_LIB=$R/gnark-icicle_amd/libgnark_mi355x_alt3.so"
AB_TIMEOUT=120 bash tools/ab_run.sh gpurun_out/r06g_fixup_ab.txt 3 "" "$ALT" -- python3 tools/msm_only.py --logn 20 --reps 10 || exit 1
AB_TIMEOUT=120 bash tools/ab_run.sh gpurun_out/r06g_fixup_ab.txt 2 "" "$ALT" -- python3 tools/msm_only.py --logn 20 --reps 5 --g2 || exit 1
AB_TIMEOUT=200 bash tools/ab_run.sh gpurun_out/r06g_fixup_ab.txt 2 "" "$ALT" -- python3 tools/g16_only.py --logn 24 --reps 3 || exit 1
AB_TIMEOUT=300 bash tools/ab_run.sh gpurun_out/r06g_fixup_ab.txt 2 "" "$ALT" -- python3 tools/g16_only.py --logn 24 --reps 3 --precompute || exit 1
AB_TIMEOUT=150 bash tools/ab_run.sh gpurun_out/r06g_bench_ab.txt 2 "" "$ALT" -- python3 bench.py --steps 20 --warmup 5 --no-secondary --no-cpu-baseline > /dev/null || exit 1
python3 - <<'PY'
import json
for l in open("gpurun_out/r06g_bench_ab.txt"):
    tag, js = l.split(" | ", 1)
    d = json.loads(js); r = d["roofline"]
    print(tag[:40], d["value"], d["ms_per_step"], r["avg_launch_ms"], r.get("timing_source"), d["kernel_avg_ms"].get("msm_fixup"))
PY
