#!/bin/bash
# r06e: the driver's exact bench command, then the same command under rocprofv3 --kernel-trace --stats
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out && export TMPDIR=/tmp
T=${1:-r06e}
timeout -k 10 900 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -30 gpurun_out/${T}_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/${T}_bench.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], r['avg_launch_ms'], r['frac'], r['timing_source'])"
timeout -k 10 1000 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof -o prof -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${T}_profbench.json 2> gpurun_out/${T}_prof.err || { tail -30 gpurun_out/${T}_prof.err; exit 1; }
TR=$(find gpurun_out/${T}_prof -name "*kernel_trace.csv" | head -1)
ST=$(find gpurun_out/${T}_prof -name "*kernel_stats.csv" | head -1)
python3 tools/prof_trace_summary.py "$TR" > gpurun_out/${T}_trace_summary.txt
python3 tools/prof_trace_summary.py "$TR" --match accum_seg_ch --grid 0 --skip 8 --take 20 | tee gpurun_out/${T}_bench_launches.txt
python3 tools/prof_summary.py "$ST" > gpurun_out/${T}_rocprof_summary.txt
head -8 gpurun_out/${T}_trace_summary.txt
python3 -c "import json; d=json.load(open('gpurun_out/${T}_profbench.json')); r=d['roofline']; print('under rocprof:', d['value'], d['ms_per_step'], r['avg_launch_ms'], r['frac'], r['timing_source'])"
gzip -f "$TR"
