#!/bin/bash
# r05b: default bench MSM line with the library's load-time hardware-queue default
# (nothing set by the bench), against an explicit 4-queue run, plus a kernel trace
# of the step loop with the variable unset.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r05b && export TMPDIR=/tmp
O=gpurun_out/r05b
unset GPU_MAX_HW_QUEUES
for i in 1 2; do
  timeout -k 10 240 python -u bench.py --no-secondary --steps 30 > $O/bench_default_$i.json 2>> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
done
GPU_MAX_HW_QUEUES=4 timeout -k 10 240 python -u bench.py --no-secondary --steps 30 > $O/bench_q4.json 2>> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o trace -- python3 bench.py --no-secondary --no-cpu-baseline --steps 20 > $O/trace_bench.json 2> $O/trace.err || { tail -30 $O/trace.err; exit 1; }
python3 tools/msm_timeline.py $(ls $O/trace/*kernel_trace.csv $O/trace/*/*kernel_trace.csv 2>/dev/null | head -1) 16 > $O/msm_loop_timeline_libdefault.txt
find $O/trace -name "*.csv" -delete
for f in $O/bench_default_1.json $O/bench_default_2.json $O/bench_q4.json; do python3 -c "import json,sys; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'], d['hip_hw_queues'])"; done
head -3 $O/msm_loop_timeline_libdefault.txt
