#!/bin/bash
# r05f: MSM parity with the accumulation-chain default, FETCH_SIZE calibration of
# the 64-B gather (tools/microbench/gather), then the final kernels' counters:
# VALU passes over the 2^20 G1 MSM and the 2^24 NTT, FETCH / WRITE over the MSM,
# and the kernel stats of the default bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-r05f}
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_msm_gpu.py tests/test_golden_gpu.py > gpurun_out/${T}_msm_tests.txt 2>&1 || { tail -30 gpurun_out/${T}_msm_tests.txt; exit 1; }
tail -1 gpurun_out/${T}_msm_tests.txt
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${T}_gather -o pmc -- tools/microbench/gather > gpurun_out/${T}_gather.out 2>&1 || { tail -20 gpurun_out/${T}_gather.out; exit 1; }
python3 - <<PY > gpurun_out/${T}_gather_fetch.txt
import csv, glob
rows = []
for f in glob.glob("gpurun_out/${T}_gather/**/*counter_collection*.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r.get("Dispatch_Id", 0)))
print(open("gpurun_out/${T}_gather.out").read())
for r in rows:
    print(r["Kernel_Name"].split("(")[0], r["Counter_Name"], r["Counter_Value"], "KiB")
PY
cat gpurun_out/${T}_gather_fetch.txt | tail -8
bash tools/gpu_pmc.sh ${T}_valu --logn 20 --reps 5 > /dev/null || exit 1
python3 tools/pmc_valu.py gpurun_out/${T}_pmc_valu.json gpurun_out/${T}_valu_pmc1 gpurun_out/${T}_valu_pmc2 > /dev/null || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/${T}_pmc_valu.json')); print({k: v for k, v in d.items() if 'accum' in k})"
PROG=tools/ntt_only.py bash tools/gpu_pmc.sh ${T}_ntt --logn 24 --reps 2 > /dev/null || exit 1
python3 tools/pmc_valu.py gpurun_out/${T}_ntt_pmc_valu.json gpurun_out/${T}_ntt_pmc1 gpurun_out/${T}_ntt_pmc2 > /dev/null || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/${T}_ntt_pmc_valu.json')); print({k: v for k, v in d.items() if 'ntt' in k})"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${T}_f -o pmc -- python3 tools/msm_only.py --logn 20 --reps 5 > /dev/null 2> gpurun_out/${T}_f.err || { tail -20 gpurun_out/${T}_f.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${T}_w -o pmc -- python3 tools/msm_only.py --logn 20 --reps 5 > /dev/null 2> gpurun_out/${T}_w.err || { tail -20 gpurun_out/${T}_w.err; exit 1; }
python3 tools/pmc_traffic.py gpurun_out/${T}_f gpurun_out/${T}_w gpurun_out/${T}_pmc_traffic.json > /dev/null || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/${T}_pmc_traffic.json')); print('accum traffic', {k: v for k, v in d.items() if 'accum' in k})"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof -o prof -- python3 bench.py --no-cpu-baseline --no-secondary > gpurun_out/${T}_profbench.json 2> gpurun_out/${T}_prof.err || { tail -30 gpurun_out/${T}_prof.err; exit 1; }
python3 tools/prof_summary.py $(ls gpurun_out/${T}_prof/*kernel_stats.csv gpurun_out/${T}_prof/*/*kernel_stats.csv 2>/dev/null | head -1) > gpurun_out/${T}_rocprof_summary.txt
head -8 gpurun_out/${T}_rocprof_summary.txt
find gpurun_out/${T}_* -name "*.csv" -size +5M -delete
