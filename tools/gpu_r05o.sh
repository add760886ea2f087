#!/bin/bash
# r05o: MSM / Groth16 GPU tests with the staged pass-1 scatter, then same-box A/B
# (GM_MSM_S1_STAGED=0 vs default) of the bench MSM line and of 2^24 host-input proves.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05o; mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_msm_gpu.py tests/test_golden_gpu.py tests/test_groth16_gpu.py tests/test_configs_full.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for rep in 1 2 3; do
  for v in 0 1; do
    GM_MSM_S1_STAGED=$v timeout -k 10 300 python3 bench.py --no-secondary --no-cpu-baseline > $O/b_${v}_$rep.json 2>> $O/b.err || { tail -20 $O/b.err; exit 1; }
    python3 -c "
import json
d=json.loads(open('$O/b_${v}_$rep.json').read().strip().splitlines()[-1])
print('s1_staged=$v rep=$rep', d['value'], d['ms_per_step'], d['kernel_avg_ms'])" | tee -a $O/ab.txt
  done
done
for rep in 1 2; do
  for v in 0 1; do
    echo "== g16 s1_staged=$v rep $rep" >> $O/ab.txt
    GM_MSM_S1_STAGED=$v timeout -k 10 300 python3 tools/g16_host_trace.py device >> $O/ab.txt 2>> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  done
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o prof -- python3 tools/msm_only.py --logn 20 --reps 5 > /dev/null 2> $O/prof.err || { tail -20 $O/prof.err; exit 1; }
python3 tools/prof_summary.py $(ls $O/prof/*kernel_stats.csv $O/prof/*/*kernel_stats.csv 2>/dev/null | head -1) > $O/msm_only_summary.txt
find $O/prof -name "*trace.csv" -delete
cat $O/ab.txt; head -14 $O/msm_only_summary.txt
