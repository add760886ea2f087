#!/bin/bash
# r05m: MSM GPU tests with the LDS-staged point conversion, then a same-box A/B of the bench
# MSM lines (GM_MSM_CONVERT_LDS=0 vs default), alternating fresh processes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05m; mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_msm_gpu.py tests/test_golden_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for rep in 1 2 3; do
  for v in 0 1; do
    GM_MSM_CONVERT_LDS=$v timeout -k 10 300 python3 bench.py --g16-logn "" --g16-plain "" --no-cpu-baseline > $O/b_${v}_$rep.json 2>> $O/b.err || { tail -20 $O/b.err; exit 1; }
    python3 -c "
import json,sys
d=json.loads(open('$O/b_${v}_$rep.json').read().strip().splitlines()[-1])
s=d.get('secondary',{})
print('lds=$v rep=$rep', d['value'], d['ms_per_step'], {k: v.get('mpoints_per_s', v.get('ms')) for k, v in s.get('msm', {}).items()})" | tee -a $O/ab.txt
  done
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o prof -- python3 tools/msm_only.py --logn 20 --reps 5 > /dev/null 2> $O/prof.err || { tail -20 $O/prof.err; exit 1; }
python3 tools/prof_summary.py $(ls $O/prof/*kernel_stats.csv $O/prof/*/*kernel_stats.csv 2>/dev/null | head -1) > $O/msm_only_summary.txt && cat $O/msm_only_summary.txt
find $O/prof -name "*trace.csv" -delete
