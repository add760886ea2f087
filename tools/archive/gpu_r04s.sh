#!/bin/bash
# r04s: kernel + memory-copy trace of 2^24 host-input proves in a fresh process
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-r04s}
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/${T}_kt -o kt -- python3 -u tools/g16_host_trace.py > gpurun_out/${T}.log 2>&1 || { tail -30 gpurun_out/${T}.log; exit 1; }
cat gpurun_out/${T}.log | grep prove
ls -la gpurun_out/${T}_kt/ gpurun_out/${T}_kt/*/ 2>/dev/null | head
F=$(ls gpurun_out/${T}_kt/*kernel_trace.csv gpurun_out/${T}_kt/*/*kernel_trace.csv 2>/dev/null | head -1)
python3 tools/g16_timeline.py $F --all > gpurun_out/${T}_timeline.txt; tail -5 gpurun_out/${T}_timeline.txt
M=$(ls gpurun_out/${T}_kt/*memory_copy_trace.csv gpurun_out/${T}_kt/*/*memory_copy_trace.csv 2>/dev/null | head -1)
python3 - "$M" "$F" <<'PY' > gpurun_out/${T}_copies.txt
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
k = list(csv.DictReader(open(sys.argv[2])))
k.sort(key=lambda r: int(r["Start_Timestamp"]))
# last prove: from the last-but-one digits kernel of the wire plan
dig = [int(r["Start_Timestamp"]) for r in k if "k_msm_digits" in r["Kernel_Name"]]
t0 = dig[-2] if len(dig) >= 2 else int(k[0]["Start_Timestamp"])
print(list(rows[0].keys()))
for r in sorted(rows, key=lambda r: int(r["Start_Timestamp"])):
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if s >= t0 - 60_000_000:
        print("%9.3f %8.3f %s %s" % ((s - t0) / 1e6, (e - s) / 1e6, r.get("Direction", r.get("Operation", "")), r.get("Size", r.get("Bytes", ""))))
PY
head -60 gpurun_out/${T}_copies.txt
find gpurun_out/${T}_kt -name "*.csv" -size +20M -delete
