#!/bin/bash
# r05ab (experiment): async MSM plan on the high-priority slot stream, accumulation / reduction /
# readback on a second per-slot stream (GM_MSM_PLAN_FIRST=1, GM_MSM_ACC_PRIO 0 = least, 1 = greatest).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05ab; mkdir -p $O && export TMPDIR=/tmp
GM_MSM_PLAN_FIRST=1 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_msm_gpu.py -k "async or bench_input" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  for v in "0 0" "1 0" "1 1"; do
    set -- $v
    GM_MSM_PLAN_FIRST=$1 GM_MSM_ACC_PRIO=$2 timeout -k 10 300 python3 bench.py --no-secondary --no-cpu-baseline > $O/b.json 2>> $O/b.err || { tail -20 $O/b.err; exit 1; }
    python3 -c "
import json
d=json.loads(open('$O/b.json').read().strip().splitlines()[-1])
print('plan_first=$1 acc_prio=$2 rep=$rep', d['value'], d['ms_per_step'])" | tee -a $O/ab.txt
  done
done
grep -m1 priorities $O/b.err || true
GM_MSM_PLAN_FIRST=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o tr -- python3 bench.py --no-secondary --no-cpu-baseline --steps 20 > /dev/null 2>> $O/tr.err || { tail -30 $O/tr.err; exit 1; }
python3 tools/msm_timeline.py $(ls $O/tr/*kernel_trace.csv $O/tr/*/*kernel_trace.csv 2>/dev/null | head -1) 16 > $O/timeline.txt
find $O/tr -name "*.csv" -delete
head -1 $O/timeline.txt
