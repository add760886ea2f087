#!/bin/bash
# r05ag: accumulation launches timed by their own start / end (hipExtLaunchKernelGGL events): MSM tests,
# the default bench line and the rocprofv3 kernel stats of the same command.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05ag; mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_msm_gpu.py tests/test_groth16_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python3 bench.py --no-secondary --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o prof -- python3 bench.py --no-cpu-baseline --no-secondary > $O/profbench.json 2> $O/prof.err || { tail -30 $O/prof.err; exit 1; }
python3 tools/prof_summary.py $(ls $O/prof/*kernel_stats.csv $O/prof/*/*kernel_stats.csv 2>/dev/null | head -1) > $O/rocprof_summary.txt
find $O/prof -name "*trace.csv" -delete
for f in bench profbench; do python3 -c "
import json
d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1])
r=d['roofline']
print('$f', d['value'], d['ms_per_step'], 'acc ms', r['avg_launch_ms'], 'frac', r['frac'], 'int_alu', r['int_alu']['frac'], 'iso', r['isolated'])"; done
head -4 $O/rocprof_summary.txt
