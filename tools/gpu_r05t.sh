#!/bin/bash
# r05t (experiment): CU-split async MSMs (GM_MSM_CU_SIDE=k: sort / reduction on every k-th CU,
# accumulation on the rest) against the default, bench A/B + traces.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05t; mkdir -p $O && export TMPDIR=/tmp
GM_MSM_CU_SIDE=8 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_msm_gpu.py -k "async or bench_input" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for rep in 1 2; do
  for v in 0 8 16; do
    GM_MSM_CU_SIDE=$v timeout -k 10 300 python3 bench.py --no-secondary --no-cpu-baseline > $O/b_${v}_$rep.json 2>> $O/b.err || { tail -20 $O/b.err; exit 1; }
    python3 -c "
import json
d=json.loads(open('$O/b_${v}_$rep.json').read().strip().splitlines()[-1])
print('cu_side=$v rep=$rep', d['value'], d['ms_per_step'], d['latency_ms'])" | tee -a $O/ab.txt
  done
done
for v in 8 16; do
  GM_MSM_CU_SIDE=$v timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr_$v -o tr -- python3 bench.py --no-secondary --no-cpu-baseline --steps 20 > /dev/null 2>> $O/tr.err || { tail -30 $O/tr.err; exit 1; }
  python3 tools/msm_timeline.py $(ls $O/tr_$v/*kernel_trace.csv $O/tr_$v/*/*kernel_trace.csv 2>/dev/null | head -1) 16 > $O/timeline_$v.txt
  find $O/tr_$v -name "*.csv" -delete
  head -1 $O/timeline_$v.txt
done
