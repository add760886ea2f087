#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 ./tools/microbench/h2d 2>&1 | tee gpurun_out/r02c_h2d.txt || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r02c_zero -o z -- python3 tools/msm_only.py --scalars zero --reps 3 > gpurun_out/r02c_zero.out 2>&1 || { tail gpurun_out/r02c_zero.out; exit 1; }
cat gpurun_out/r02c_zero.out | tail -2
python3 - <<'PY'
import csv,glob
f=glob.glob("gpurun_out/r02c_zero/**/*kernel_stats.csv",recursive=True)[0]
for r in csv.DictReader(open(f)):
    print("%-60s %6s %10.1f us avg" % (r["Name"][:60], r["Calls"], float(r["AverageNs"])/1e3))
PY
