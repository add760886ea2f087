#!/bin/bash
# r05n: kernel trace of the bench's pipelined MSM loop with the LDS conversion.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05n; mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o trace -- python3 bench.py --no-secondary --no-cpu-baseline --steps 20 > $O/trace_bench.json 2> $O/trace.err || { tail -30 $O/trace.err; exit 1; }
python3 tools/msm_timeline.py $(ls $O/trace/*kernel_trace.csv $O/trace/*/*kernel_trace.csv 2>/dev/null | head -1) 16 > $O/msm_loop_timeline.txt
find $O/trace -name "*.csv" -delete
cat $O/msm_loop_timeline.txt
