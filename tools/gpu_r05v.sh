#!/bin/bash
# r05v: whole -m gpu suite with per-slot low-priority reduction streams, then the bench A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05v; mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for rep in 1 2 3; do
  for v in 0 1; do
    GM_MSM_RED_STREAM=$v timeout -k 10 300 python3 bench.py --no-secondary --no-cpu-baseline > $O/b_${v}_$rep.json 2>> $O/b.err || { tail -20 $O/b.err; exit 1; }
    python3 -c "
import json
d=json.loads(open('$O/b_${v}_$rep.json').read().strip().splitlines()[-1])
print('red_stream=$v rep=$rep', d['value'], d['ms_per_step'], d['latency_ms'], d['roofline']['avg_launch_ms'])" | tee -a $O/ab.txt
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o tr -- python3 bench.py --no-secondary --no-cpu-baseline --steps 20 > /dev/null 2>> $O/tr.err || { tail -30 $O/tr.err; exit 1; }
python3 tools/msm_timeline.py $(ls $O/tr/*kernel_trace.csv $O/tr/*/*kernel_trace.csv 2>/dev/null | head -1) 16 > $O/timeline.txt
find $O/tr -name "*.csv" -delete
head -1 $O/timeline.txt
